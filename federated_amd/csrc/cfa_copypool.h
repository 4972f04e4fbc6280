// cfa_copypool.h — fork-join pool of host threads for memcpy lists (host only, no HIP).
//
// The drop-in host mix (cfa_hostmix.cpp) packs each chunk of the local and neighbour models
// into pinned staging with a few host threads, and unpacks each chunk's result the same way
// (SURVEY §8 f2). The reference calls that mix from one Python thread per simulated device
// (TF2 CIFAR100_dataset/federated_learning_keras_consensus_FL_threads_CIFAR100.py:674-681, mixing
// at MNIST_dataset/consensus/consensus_v3.py:144-157), so the pool is entered concurrently.
//
// Protocol (one run at a time; a caller that finds the pool busy copies on its own thread):
//   - run() owns the job list for the run (copied into pool storage), resets the claim and the
//     completion counters, then publishes ONE atomic word  state = gen << 8 | helpers  (open).
//   - A worker takes its part in a run from a single load of that word: worker `id` may help
//     generation g when it observes g open and id < helpers(g). The generation and the helper
//     count can never come from two different runs.
//   - Joining is a claim: the worker enters (active += 1), then re-reads the word and drains jobs
//     only if it still holds exactly the open word it observed; otherwise it leaves (active -= 1)
//     without touching the job list.
//   - run() drains jobs itself, waits until every job has completed, then CLOSES the run (state
//     = gen << 8 | 0) and waits until no worker is active. Both the claim and the close are a
//     store followed by a load of the other side's word (sequentially consistent), so either the
//     worker sees the run closed and leaves, or run() sees the worker active and waits for it: no
//     worker touches a job list after its run returned. Late workers simply miss the run, so run()
//     never waits for a helper that was not needed (with more helpers than free cores, waiting for
//     every helper to wake had cost a scheduling round per run).
//   - run()'s waits are bounded: past `timeout` the pool is marked broken and the run abandoned:
//     no job is handed out any more (the claim counter is pushed past the list) and the run is
//     closed, then run() waits (up to `straggler_timeout`, 10 minutes) until every helper still
//     inside a copy has left, so that when it returns false no helper writes the caller's buffers
//     any more and the caller may free them. Every later run copies on its caller's thread. Only
//     if a helper is still inside a copy after `straggler_timeout` (a copy that cannot finish)
//     does run() return with it there; the caller must then keep its buffers alive
//     (`stragglers()` > 0).
// Workers spin (pausing, then yielding the core) for ~50 us after each run before parking on a
// condition variable, so the runs of one pipelined call (one per chunk, tens of microseconds
// apart) do not pay a futex wake-up each.
#ifndef CFA_COPYPOOL_H
#define CFA_COPYPOOL_H

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace cfa {

struct Copy {
  void* dst;
  const void* src;
  size_t bytes;
};

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

class CopyPool {
 public:
  static constexpr int kMaxThreads = 64;  // caller + 63 helpers; helpers fit the state's low byte

  CopyPool() = default;
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;

  // Stops and joins the workers (a broken pool's straggler is joined after its copy finishes, so
  // the buffers of a timed-out run must outlive the pool; the library's process-wide pool is
  // never destroyed).
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_.store(true, std::memory_order_relaxed);
      publish(0);
    }
    cv_.notify_all();
    for (std::thread& t : workers_)
      if (t.joinable()) t.join();
  }

  // Copies every job, on up to `threads` threads (the caller included). Returns false only when
  // the jobs or the helpers did not finish within `timeout` (the pool is then broken; see above).
  bool run(const Copy* jobs, size_t njobs, int threads,
           std::chrono::nanoseconds timeout = std::chrono::seconds(30),
           std::chrono::nanoseconds straggler_timeout = std::chrono::minutes(10)) {
    if (njobs == 0) return true;
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    const int want = int(std::min<size_t>(size_t(std::clamp(threads, 1, kMaxThreads)), njobs));
    if (!busy.owns_lock() || want <= 1 || broken_.load(std::memory_order_relaxed)) {
      for (size_t i = 0; i < njobs; ++i) std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
      return true;
    }
    const int helpers = want - 1;
    ensure(helpers);
    jobs_.assign(jobs, jobs + njobs);
    next_.store(0, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);  // under the lock: a parking worker cannot miss it
      publish(helpers);                    // release: jobs_, next_, done_ happen-before
    }
    cv_.notify_all();
    drain(jobs_);
    const auto t0 = std::chrono::steady_clock::now();
    if (!wait([&] { return done_.load(std::memory_order_acquire) == njobs; }, t0, timeout))
      return abandon(straggler_timeout);
    close();
    if (!wait([&] { return active_.load(std::memory_order_seq_cst) == 0; }, t0, timeout))
      return abandon(straggler_timeout);
    return true;
  }

  bool broken() const { return broken_.load(std::memory_order_relaxed); }
  // Helpers still inside a copy of an abandoned run (0 once run() has returned, unless a copy
  // outlived straggler_timeout).
  int stragglers() const { return active_.load(std::memory_order_acquire); }
  int workers() const { return int(workers_.size()); }
  uint64_t generation() const { return state_.load(std::memory_order_relaxed) >> 8; }

 private:
  // Caller holds mu_. Bumps the generation and sets the helper count in one store.
  void publish(int helpers) {
    const uint64_t gen = (state_.load(std::memory_order_relaxed) >> 8) + 1;
    state_.store(gen << 8 | uint64_t(helpers), std::memory_order_seq_cst);
  }

  // The current run takes no more helpers: same generation, helper count 0 (a worker waiting for
  // a new generation does not wake for it; a joining worker re-reads the word and leaves).
  void close() {
    const uint64_t s = state_.load(std::memory_order_relaxed);
    state_.store(s & ~uint64_t(0xff), std::memory_order_seq_cst);
  }

  // Spins (then yields) until pred(); past `timeout` marks the pool broken and returns false:
  // stragglers may still read jobs_ and bump the counters, and a broken pool never touches them
  // again (every later run copies on its caller's thread).
  template <class Pred>
  bool wait(Pred pred, std::chrono::steady_clock::time_point t0, std::chrono::nanoseconds timeout) {
    for (long spin = 0; !pred(); ++spin) {
      if (spin < 4096) {
        cpu_relax();
        continue;
      }
      std::this_thread::yield();
      if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > timeout) {
        broken_.store(true, std::memory_order_relaxed);
        return false;
      }
    }
    return true;
  }

  // The run timed out (the pool is already marked broken): hand out no more jobs, take no more
  // helpers, and wait until the helpers inside a copy have left. Returns false (the run failed).
  bool abandon(std::chrono::nanoseconds straggler_timeout) {
    next_.store(size_t(1) << 62, std::memory_order_seq_cst);  // every later claim is past the list
    close();
    const auto t1 = std::chrono::steady_clock::now();
    while (active_.load(std::memory_order_seq_cst) != 0 &&
           std::chrono::steady_clock::now() - t1 < straggler_timeout)
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    return false;
  }

  // Caller holds run_mu_, so the generation cannot move while workers are created.
  void ensure(int n) {
    std::lock_guard<std::mutex> g(mu_);
    const uint64_t gen = state_.load(std::memory_order_relaxed) >> 8;
    while (int(workers_.size()) < n) {
      const int id = int(workers_.size());
      workers_.emplace_back([this, id, gen] { loop(id, gen); });
    }
  }

  void drain(const std::vector<Copy>& jobs) {
    for (size_t i = next_.fetch_add(1, std::memory_order_relaxed); i < jobs.size();
         i = next_.fetch_add(1, std::memory_order_relaxed)) {
      std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
      done_.fetch_add(1, std::memory_order_release);
    }
  }

  // One load of state_ whose generation differs from `seen`: spin (pausing, then yielding the
  // core, so a caller sharing it with idle workers is not held up), then park.
  uint64_t await(uint64_t seen) {
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0;; ++spin) {
      const uint64_t s = state_.load(std::memory_order_acquire);
      if ((s >> 8) != seen) return s;
      if ((spin & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50)) {
        std::unique_lock<std::mutex> g(mu_);
        uint64_t w = 0;
        cv_.wait(g, [&] {
          w = state_.load(std::memory_order_acquire);
          return (w >> 8) != seen;
        });
        return w;
      }
      if (spin < 256) cpu_relax();
      else std::this_thread::yield();
    }
  }

  void loop(int id, uint64_t seen) {
    for (;;) {
      const uint64_t s = await(seen);
      seen = s >> 8;
      if (stop_.load(std::memory_order_relaxed)) return;
      if (id >= int(s & 0xff)) continue;  // not a helper of generation `seen` (or already closed)
      active_.fetch_add(1, std::memory_order_seq_cst);
      if (state_.load(std::memory_order_seq_cst) == s) drain(jobs_);  // still open: jobs_ is stable
      active_.fetch_sub(1, std::memory_order_release);
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
  std::vector<Copy> jobs_;  // the current run's job list (pool-owned: outlives the caller's)
  std::atomic<size_t> next_{0}, done_{0};
  std::atomic<int> active_{0};
  std::atomic<uint64_t> state_{0};  // gen << 8 | helpers (0 once the run is closed)
  std::atomic<bool> stop_{false}, broken_{false};
};

}  // namespace cfa

#endif  // CFA_COPYPOOL_H
