// copypool_stress.cpp — CPU stress test of the host copy pool (federated_amd/csrc/cfa_copypool.h).
//
// Built without HIP by tests/test_copypool.py, plain and under ThreadSanitizer. The pool is the
// fork-join pool behind cfa_host_mix_f32, which the reference enters from one
// Python thread per device (TF2 CIFAR100_dataset/...FL_threads_CIFAR100.py:674-681). Round 2's
// pool read the generation and the helper count as two loads, so a worker idle in one run could
// double-count the next when the helper count changed between runs; this test alternates helper
// counts 1/3/7/15 with random job counts (often fewer jobs than threads, so the effective helper
// count varies too) and checks, after every run:
//   - every destination byte equals its source (no job skipped or half-done when run returns);
//   - bytes outside the jobs' ranges are untouched;
//   - the caller then rewrites the destination at once, so a worker still writing after run()
//     returned is a data race ThreadSanitizer reports (and a content error the next check sees).
// Then several caller threads enter one pool at once (the busy pool falls back to the caller's
// thread), and a zero timeout exercises the broken-pool path.
//
// usage: copypool_stress RUNS SEED
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "cfa_copypool.h"

namespace {

constexpr size_t kArena = size_t(1) << 13;  // bytes per source / destination arena

int failures = 0;

void fail(const char* what, long run) {
  if (failures++ < 10) std::fprintf(stderr, "FAIL run %ld: %s\n", run, what);
}

struct Arena {
  std::vector<unsigned char> src, dst;
  Arena() : src(kArena), dst(kArena) {}
};

// One run: random disjoint ranges of `a.dst`, copied from the same offsets of `a.src`, then
// checked and overwritten by the calling thread.
void one_run(cfa::CopyPool& pool, Arena& a, std::mt19937_64& rng, long r, int threads) {
  const unsigned char tag = static_cast<unsigned char>(r * 131 + 7);
  std::uniform_int_distribution<int> njobs_d(1, (r % 5 == 0) ? 2 : 48);
  const int njobs = njobs_d(rng);
  std::vector<cfa::Copy> jobs;
  std::vector<std::pair<size_t, size_t>> ranges;
  size_t off = 0;
  for (int j = 0; j < njobs && off < kArena; ++j) {
    std::uniform_int_distribution<size_t> gap_d(0, 8), len_d(1, 128);
    off += gap_d(rng);
    const size_t len = std::min(len_d(rng), kArena - std::min(off, kArena));
    if (len == 0) break;
    for (size_t i = 0; i < len; ++i) a.src[off + i] = static_cast<unsigned char>(tag + i * 3 + j);
    jobs.push_back({a.dst.data() + off, a.src.data() + off, len});
    ranges.push_back({off, off + len});
    off += len;
  }
  std::memset(a.dst.data(), 0xA5, kArena);
  if (!pool.run(jobs.data(), jobs.size(), threads)) fail("timeout", r);
  size_t pos = 0;
  for (const auto& [x, y] : ranges) {
    for (size_t i = pos; i < x; ++i)
      if (a.dst[i] != 0xA5) { fail("byte outside the jobs written", r); break; }
    if (std::memcmp(a.dst.data() + x, a.src.data() + x, y - x) != 0) fail("job not copied", r);
    pos = y;
  }
  for (size_t i = pos; i < kArena; ++i)
    if (a.dst[i] != 0xA5) { fail("byte past the jobs written", r); break; }
  std::memset(a.dst.data(), 0x5A, kArena);  // a late helper write races with this
}

}  // namespace

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  auto t0 = std::chrono::steady_clock::now();
  const long runs = argc > 1 ? std::atol(argv[1]) : 100000;
  const unsigned long long seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
  static const int helper_cycle[] = {1, 3, 7, 15};

  {  // phase 1: one caller, helper counts alternating 1/3/7/15
    cfa::CopyPool pool;
    Arena a;
    std::mt19937_64 rng(seed);
    for (long r = 0; r < runs && failures == 0; ++r) one_run(pool, a, rng, r, helper_cycle[r % 4] + 1);
    if (pool.generation() == 0) fail("pool never published a run", -1);
    if (pool.broken()) fail("pool broken after phase 1", -1);
    std::printf("phase 1: %ld runs, %d workers, generation %llu (%.1f s)\n", runs, pool.workers(),
                static_cast<unsigned long long>(pool.generation()), seconds_since(t0));
    t0 = std::chrono::steady_clock::now();
  }
  {  // phase 2: four callers at once on one pool (each run either owns the pool or copies alone)
    cfa::CopyPool pool;
    std::vector<std::thread> callers;
    const long per = std::max(1L, runs / 8);
    for (int c = 0; c < 4; ++c)
      callers.emplace_back([&pool, per, seed, c] {
        Arena a;
        std::mt19937_64 rng(seed * 1000 + c);
        for (long r = 0; r < per; ++r) one_run(pool, a, rng, r, helper_cycle[(r + c) % 4] + 1);
      });
    for (std::thread& t : callers) t.join();
    std::printf("phase 2: 4 callers x %ld runs, generation %llu (%.1f s)\n", per,
                static_cast<unsigned long long>(pool.generation()), seconds_since(t0));
  }
  {  // phase 3: a zero timeout may break the pool; later runs must still be complete
    // 16 jobs of 4 MiB on 8 threads: helpers are still inside a copy when the caller, done with its
    // own share, finds the zero timeout spent. The buffers are declared before the pool, so they
    // outlive the stragglers the pool's destructor joins.
    constexpr size_t kBig = size_t(4) << 20;
    std::vector<unsigned char> big_src(16 * kBig, 1), big_dst(16 * kBig, 0);
    Arena b;
    cfa::CopyPool pool;
    std::mt19937_64 rng(seed + 99);
    std::vector<cfa::Copy> jobs;
    for (size_t o = 0; o < big_src.size(); o += kBig) jobs.push_back({big_dst.data() + o, big_src.data() + o, kBig});
    const bool ok = pool.run(jobs.data(), jobs.size(), 8, std::chrono::nanoseconds(0));
    // a timed-out run returns only once no helper is inside a copy of its buffers any more
    if (!ok && pool.stragglers() != 0) fail("timed-out run returned with helpers still copying", -1);
    // meanwhile the pool must serve complete runs on other buffers
    for (long r = 0; r < 200; ++r) one_run(pool, b, rng, r, 4);
    std::printf("phase 3: zero-timeout run %s, pool %s\n", ok ? "completed" : "timed out",
                pool.broken() ? "broken (serial fallback)" : "healthy");
    if (!ok && !pool.broken()) fail("timeout without marking the pool broken", -1);
  }
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
