// Stress of the host lane's pump (federated_amd/csrc/cfa_lane.cpp) in host mode, built without
// HIP (the few HIP and libcfa symbols the GPU mode calls are stubbed below and must never run),
// plainly and under ThreadSanitizer (tests/test_lane_pump_native.py).
//
// A producer thread plays the sending rank: for each round it fills the chunks of one parity of a
// "segment" and raises the READY word chunk by chunk, with random pauses, after waiting for the
// consumer's ACK of the round two back (the lane's back-pressure). The consumer (this thread) is
// the receiving rank: it submits the round's operations to the pump (wait READY, copy the chunk
// out, publish a mark per group of chunks; at the end raise the ACK), waits for the group marks in
// order, checks each group's rows as soon as its mark is published, then waits for the round.
// Every round's rows carry the round number, so a copy from the wrong parity or too early shows.
// Then: a round whose word never comes times out (sticky), and destroy interrupts a pending wait.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "cfa_engine.h"

// ---- stubs: the GPU mode's calls (never reached in host mode) ----
extern "C" hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t) { std::abort(); }
extern "C" hipError_t hipEventRecord(hipEvent_t, hipStream_t) { std::abort(); }
extern "C" hipError_t hipSetDevice(int) { std::abort(); }
extern "C" const char* hipGetErrorString(hipError_t) { return "stub"; }
extern "C" int cfa_stream_signal(unsigned*, unsigned, void*) { std::abort(); }
static thread_local char g_err[512];
extern "C" void cfa_internal_set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg ? msg : ""); }
extern "C" const char* cfa_last_error(void) { return g_err; }

static void fail(const char* what) {
  printf("FAIL %s (%s)\n", what, g_err);
  std::exit(1);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 2000;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1;
  const int chunks = 12, chunk_elems = 256, groups = 3;
  std::vector<float> seg(2 * chunks * chunk_elems);   // two parities
  std::vector<float> dst(chunks * chunk_elems);
  unsigned words[32] = {0};  // READY at 0, ACK at 16
  unsigned* ready = &words[0];
  unsigned* ack = &words[16];

  void* pump = nullptr;
  if (cfa_lane_pump_create(&pump, nullptr, 0, 1) != CFA_OK) fail("create");

  std::atomic<bool> producer_error{false};
  std::thread producer([&] {
    std::mt19937 rng(seed);
    for (int r = 0; r < rounds; ++r) {
      if (r >= 2) {  // the consumer has drained round r - 2 from this parity
        const auto t0 = std::chrono::steady_clock::now();
        while (static_cast<int>(__atomic_load_n(ack, __ATOMIC_ACQUIRE) - (unsigned)(r - 1)) < 0) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) { producer_error = true; return; }
          std::this_thread::yield();
        }
      }
      float* par = seg.data() + (r & 1) * chunks * chunk_elems;
      for (int k = 0; k < chunks; ++k) {
        for (int i = 0; i < chunk_elems; ++i) par[k * chunk_elems + i] = (float)(r * 1000 + k);
        __atomic_store_n(ready, (unsigned)(r * chunks + k + 1), __ATOMIC_RELEASE);
        if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
      }
    }
  });

  std::vector<cfa_lane_op> ops(chunks + 1);
  for (int r = 0; r < rounds; ++r) {
    const float* par = seg.data() + (r & 1) * chunks * chunk_elems;
    for (int k = 0; k < chunks; ++k) {
      cfa_lane_op& op = ops[k];
      std::memset(&op, 0, sizeof(op));
      op.wait_word = ready;
      op.wait_value = (unsigned)(r * chunks + k + 1);
      op.dst = dst.data() + k * chunk_elems;
      op.src = par + k * chunk_elems;
      op.bytes = chunk_elems * sizeof(float);
      op.mark = ((k + 1) % (chunks / groups) == 0) ? k + 1 : 0;
    }
    std::memset(&ops[chunks], 0, sizeof(cfa_lane_op));
    ops[chunks].signal_word = ack;
    ops[chunks].signal_value = (unsigned)(r + 1);
    if (cfa_lane_pump_submit(pump, ops.data(), chunks + 1, 10000000) != CFA_OK) fail("submit");
    for (int g = 1; g <= groups; ++g) {
      const int mark = g * (chunks / groups);
      if (cfa_lane_pump_wait(pump, mark, 30000000) != CFA_OK) fail("wait mark");
      for (int k = mark - chunks / groups; k < mark; ++k)  // the group's rows, checked at its mark
        for (int i = 0; i < chunk_elems; i += 37)
          if (dst[k * chunk_elems + i] != (float)(r * 1000 + k)) {
            printf("FAIL round %d chunk %d: %f\n", r, k, dst[k * chunk_elems + i]);
            return 1;
          }
    }
    if (cfa_lane_pump_wait(pump, -1, 30000000) != CFA_OK) fail("wait round");
  }
  producer.join();
  if (producer_error) fail("producer timed out on the ack");
  printf("phase 1: %d rounds, %d chunks, %d groups\n", rounds, chunks, groups);

  // a word that never comes: the pump's wait times out, and the error is sticky
  unsigned never = 0;
  cfa_lane_op bad;
  std::memset(&bad, 0, sizeof(bad));
  bad.wait_word = &never;
  bad.wait_value = 1;
  bad.mark = 1;
  if (cfa_lane_pump_submit(pump, &bad, 1, 50000) != CFA_OK) fail("submit bad");
  if (cfa_lane_pump_wait(pump, -1, 5000000) != CFA_E_TIMEOUT) fail("timeout expected");
  if (cfa_lane_pump_submit(pump, &bad, 1, 50000) != CFA_E_TIMEOUT) fail("sticky expected");
  cfa_lane_pump_destroy(pump);

  // destroy while a wait is pending
  if (cfa_lane_pump_create(&pump, nullptr, 0, 1) != CFA_OK) fail("create 2");
  if (cfa_lane_pump_submit(pump, &bad, 1, 60000000) != CFA_OK) fail("submit 2");
  std::this_thread::sleep_for(std::chrono::milliseconds(10));
  const auto t0 = std::chrono::steady_clock::now();
  cfa_lane_pump_destroy(pump);
  if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) fail("destroy did not interrupt");
  printf("OK\n");
  return 0;
}
