// cfa_lane.cpp — the host lane's receive-side pump: one native host thread per lane.
//
// The host lane (federated_amd/hostlane.py) carries part of a sharded population's halo D2H into
// shared pinned host memory and H2D out of it, beside the xGMI links (the reference exchanges
// models as files, TF1 consensus/cfa.py:119-130; there is no device path to mirror). The sender
// raises a chunk's sequence number with a stream-ordered store after its D2H (cfa_stream_signal).
// The receiver must not enqueue the H2D before that number has arrived, and it must not wait for it
// on a GPU queue: a wait parked there holds every stream that shares its hardware queue (4 per
// process on this pool), the compute stream included.
//
// So the wait runs here, on a host thread of the lane's own: the caller submits a round's list of
// operations and returns at once; the pump walks the list, polling each operation's host word
// (acquire loads, a short spin and then 20 us sleeps, a timeout per wait), then enqueueing its copy
// on the lane's stream, its signal (the ack the sender waits for) and its event, and publishing a
// progress mark the caller can wait for (cfa_lane_pump_wait, with the GIL released when called
// through ctypes). Neither the caller's thread nor the GPU is ever blocked on the peer: the
// caller blocks only where it needs a group's rows (before that group's boundary mixes).
//
// Host mode (no GPU: the gloo tests) runs the same walk with memcpy for the copies and a host store
// for the signals, so the protocol and its timeouts are tested on CPU.
//
// A wait that times out (or a HIP error) stops the round and is sticky: every later wait and
// submit returns it. Destroy stops the thread, interrupting a wait.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char* msg);

namespace {

int lfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int lfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

bool reached(const unsigned* w, unsigned value) {
  return static_cast<int>(__atomic_load_n(w, __ATOMIC_ACQUIRE) - value) >= 0;
}

struct Pump {
  hipStream_t stream = nullptr;
  int device = 0;
  bool host_mode = false;

  std::mutex mu;
  std::condition_variable cv;
  std::vector<cfa_lane_op> ops;  // the round being walked
  long long timeout_us = 0;
  bool job = false;       // a round has been submitted and is not finished
  std::atomic<bool> stop{false};  // read by the polling loop without the lock
  int progress = 0;       // highest mark published in the current round
  int error = CFA_OK;     // sticky
  std::string message;
  std::thread worker;

  // Poll a word until it reaches value (or stop / timeout). Returns CFA_OK, CFA_E_TIMEOUT, or 1 on stop.
  int wait_word(const unsigned* w, unsigned value, long long tmo_us, std::string* why) {
    if (reached(w, value)) return CFA_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const auto spin = std::chrono::microseconds(20), limit = std::chrono::microseconds(tmo_us);
    for (unsigned i = 1;; ++i) {
      if (reached(w, value)) return CFA_OK;
      if ((i & 63) == 0) {
        if (stop.load(std::memory_order_relaxed)) return 1;
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > limit) break;
        if (dt > spin) std::this_thread::sleep_for(std::chrono::microseconds(20));
      } else {
        __builtin_ia32_pause();
      }
    }
    if (reached(w, value)) return CFA_OK;
    char buf[200];
    snprintf(buf, sizeof(buf), "timed out after %lld us waiting for word %u to reach %u", tmo_us,
             __atomic_load_n(w, __ATOMIC_ACQUIRE), value);
    *why = buf;
    return CFA_E_TIMEOUT;
  }

  // One operation: wait, copy, signal, event. Returns CFA_OK, an error code, or 1 on stop.
  int run_op(const cfa_lane_op& op, std::string* why) {
    if (op.wait_word) {
      const int rc = wait_word(op.wait_word, op.wait_value, timeout_us, why);
      if (rc != CFA_OK) return rc;
    }
    if (op.bytes) {
      if (host_mode) {
        std::memcpy(op.dst, op.src, op.bytes);
      } else {
        const hipError_t e = hipMemcpyAsync(op.dst, op.src, op.bytes, hipMemcpyDefault, stream);
        if (e != hipSuccess) { *why = std::string("hipMemcpyAsync: ") + hipGetErrorString(e); return CFA_E_HIP; }
      }
    }
    if (op.signal_word) {
      if (host_mode) {
        __atomic_store_n(op.signal_word, op.signal_value, __ATOMIC_RELEASE);
      } else if (cfa_stream_signal(op.signal_word, op.signal_value, stream) != CFA_OK) {
        *why = std::string("cfa_stream_signal: ") + cfa_last_error();
        return CFA_E_HIP;
      }
    }
    if (op.event && !host_mode) {
      const hipError_t e = hipEventRecord(static_cast<hipEvent_t>(op.event), stream);
      if (e != hipSuccess) { *why = std::string("hipEventRecord: ") + hipGetErrorString(e); return CFA_E_HIP; }
    }
    return CFA_OK;
  }

  void loop() {
    if (!host_mode) (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || (job && progress != INT_MAX); });
      if (stop) return;
      const std::vector<cfa_lane_op> todo = ops;
      lk.unlock();
      int rc = CFA_OK;
      std::string why;
      for (const cfa_lane_op& op : todo) {
        rc = run_op(op, &why);
        if (rc != CFA_OK) break;
        if (op.mark > 0) {
          std::lock_guard<std::mutex> g(mu);
          if (op.mark > progress) progress = op.mark;
          cv.notify_all();
        }
      }
      lk.lock();
      if (rc == 1) return;  // stopped
      if (rc != CFA_OK) {
        error = rc;
        message = why;
      }
      progress = INT_MAX;  // the round is over (done or failed)
      job = false;
      cv.notify_all();
    }
  }
};

}  // namespace

extern "C" int cfa_lane_pump_create(void** pump, void* stream, int device, int host_mode) {
  if (!pump) return lfail(CFA_E_INVALID, "null pump out-pointer");
  *pump = nullptr;
  Pump* p = new (std::nothrow) Pump();
  if (!p) return lfail(CFA_E_INVALID, "out of host memory");
  p->stream = static_cast<hipStream_t>(stream);
  p->device = device;
  p->host_mode = host_mode != 0;
  p->progress = INT_MAX;  // no round yet
  try {
    p->worker = std::thread([p] { p->loop(); });
  } catch (...) {
    delete p;
    return lfail(CFA_E_INVALID, "could not start the lane pump thread");
  }
  *pump = p;
  return CFA_OK;
}

extern "C" int cfa_lane_pump_submit(void* pump, const cfa_lane_op* ops, int n_ops, long long timeout_us) {
  Pump* p = static_cast<Pump*>(pump);
  if (!p) return lfail(CFA_E_INVALID, "null pump");
  if (n_ops < 0 || (n_ops > 0 && !ops)) return lfail(CFA_E_INVALID, "bad operation list (%d)", n_ops);
  if (timeout_us <= 0) return lfail(CFA_E_INVALID, "timeout_us must be positive (got %lld)", timeout_us);
  for (int i = 0; i < n_ops; ++i) {
    if (ops[i].bytes && (!ops[i].dst || !ops[i].src)) return lfail(CFA_E_INVALID, "operation %d: null copy pointer", i);
  }
  std::lock_guard<std::mutex> g(p->mu);
  if (p->error != CFA_OK) return lfail(p->error, "lane pump: %s", p->message.c_str());
  if (p->job) return lfail(CFA_E_INVALID, "lane pump: the previous round is still in progress");
  p->ops.assign(ops, ops + n_ops);
  p->timeout_us = timeout_us;
  p->progress = 0;
  p->job = true;
  p->cv.notify_all();
  return CFA_OK;
}

extern "C" int cfa_lane_pump_wait(void* pump, int mark, long long timeout_us) {
  Pump* p = static_cast<Pump*>(pump);
  if (!p) return lfail(CFA_E_INVALID, "null pump");
  if (timeout_us <= 0) return lfail(CFA_E_INVALID, "timeout_us must be positive (got %lld)", timeout_us);
  const int want = mark < 0 ? INT_MAX : mark;
  std::unique_lock<std::mutex> lk(p->mu);
  auto done = [&] { return p->error != CFA_OK || p->progress >= want; };
  // The deadline is on the steady clock; the waits are system-clock slices of at most 100 ms
  // (pthread_cond_timedwait, which ThreadSanitizer models; a clock jump costs one slice at most).
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
  while (!done()) {
    const auto now = std::chrono::steady_clock::now();
    if (now >= deadline) break;
    const auto slice = std::min<std::chrono::steady_clock::duration>(deadline - now, std::chrono::milliseconds(100));
    p->cv.wait_until(lk, std::chrono::system_clock::now() +
                             std::chrono::duration_cast<std::chrono::system_clock::duration>(slice));
  }
  if (p->error != CFA_OK) return lfail(p->error, "lane pump: %s", p->message.c_str());
  if (!done()) return lfail(CFA_E_TIMEOUT, "lane pump: mark %d not reached after %lld us (at %d)", mark, timeout_us,
                            p->progress);
  return CFA_OK;
}

extern "C" int cfa_lane_pump_destroy(void* pump) {
  Pump* p = static_cast<Pump*>(pump);
  if (!p) return CFA_OK;
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->stop.store(true);
    p->cv.notify_all();
  }
  if (p->worker.joinable()) p->worker.join();
  delete p;
  return CFA_OK;
}
