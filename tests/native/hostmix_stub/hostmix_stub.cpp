// Host emulation of what cfa_host_mix_f32 needs from HIP and from libcfa's kernels (test only).
// A stream is a worker thread running enqueued closures in order; cfa_mix_seq_f32 /
// cfa_mix_seq_div_f32 enqueue the sequential rule on the chunk's slices (kernel arguments copied at
// launch, as HIP copies them), so the pipeline's pack, "kernel" and unpack really overlap.
// cfa_host_device_pointer is the identity (host memory stands in for the mapped pinned buffers).
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cfa_engine.h"
#include "hip/hip_runtime_api.h"

struct StubStream {
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::deque<std::function<void()>> q;
  uint64_t enq = 0, done = 0;
  bool stop = false;
  std::thread worker;
  StubStream() : worker([this] { loop(); }) {}
  ~StubStream() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    worker.join();
  }
  uint64_t push(std::function<void()> fn) {
    std::lock_guard<std::mutex> g(mu);
    q.push_back(std::move(fn));
    cv.notify_all();
    return ++enq;
  }
  void loop() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        fn = std::move(q.front());
        q.pop_front();
      }
      fn();
      {
        std::lock_guard<std::mutex> g(mu);
        ++done;
      }
      done_cv.notify_all();
    }
  }
  bool reached(uint64_t t) {
    std::lock_guard<std::mutex> g(mu);
    return done >= t;
  }
  void wait(uint64_t t) {
    std::unique_lock<std::mutex> g(mu);
    done_cv.wait(g, [&] { return done >= t; });
  }
};

struct StubEvent {
  StubStream* s = nullptr;
  uint64_t ticket = 0;
};

namespace {
StubStream* default_stream() {
  static StubStream* s = new StubStream();  // never destroyed (like HIP's null stream)
  return s;
}
StubStream* resolve(hipStream_t st) { return st ? st : default_stream(); }
thread_local std::string last_error;
std::atomic<long> launches{0};

int launch(float* out, const float* local, const float* const* nbrs, const float* alphas,
           const float* divisors, int n, size_t P, void* stream) {
  if (n < 0 || (P && (!out || !local))) return CFA_E_INVALID;
  std::vector<const float*> nb(nbrs, nbrs + n);
  std::vector<float> al(alphas, alphas + n), dv;
  if (divisors) dv.assign(divisors, divisors + n);
  launches.fetch_add(1, std::memory_order_relaxed);
  resolve(static_cast<hipStream_t>(stream))->push([=] {
    for (size_t i = 0; i < P; ++i) {
      float w = local[i];
      for (int j = 0; j < n; ++j) {
        float t = nb[size_t(j)][i] - w;
        t = al[size_t(j)] * t;
        if (!dv.empty()) t = t / dv[size_t(j)];
        w = w + t;
      }
      out[i] = w;
    }
  });
  return CFA_OK;
}
}  // namespace

extern "C" {
hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned) {
  *ev = new StubEvent();
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t ev, hipStream_t st) {
  StubStream* s = resolve(st);
  ev->s = s;
  ev->ticket = s->push([] {});
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t ev) { return !ev->s || ev->s->reached(ev->ticket) ? hipSuccess : hipErrorNotReady; }
hipError_t hipEventSynchronize(hipEvent_t ev) {
  if (ev->s) ev->s->wait(ev->ticket);
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t ev) {
  delete ev;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t st) {
  StubStream* s = resolve(st);
  s->wait(s->push([] {}));
  return hipSuccess;
}

int cfa_mix_seq_f32(float* out, const float* local, const float* const* nbrs, const float* alphas, int n,
                    size_t P, void* stream) {
  return launch(out, local, nbrs, alphas, nullptr, n, P, stream);
}
int cfa_mix_seq_div_f32(float* out, const float* local, const float* const* nbrs, const float* alphas,
                        const float* divisors, int n, size_t P, void* stream) {
  return launch(out, local, nbrs, alphas, divisors, n, P, stream);
}
int cfa_host_device_pointer(const void* host, void** dev) {
  *dev = const_cast<void*>(host);
  return CFA_OK;
}
void cfa_internal_set_error(const char* msg) { last_error = msg ? msg : ""; }

// test hooks
hipStream_t stub_stream_create() { return new StubStream(); }
void stub_stream_destroy(hipStream_t s) { delete s; }
long stub_launches() { return launches.load(); }
const char* stub_last_error() { return last_error.c_str(); }
}
