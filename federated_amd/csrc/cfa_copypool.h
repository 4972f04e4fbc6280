// cfa_copypool.h — fork-join pool of host threads for memcpy lists (host only, no HIP).
//
// The drop-in host mix (cfa_hostmix.cpp) packs each chunk of the local and neighbour models
// into pinned staging with a few host threads, and unpacks each chunk's result the same way
// (SURVEY §8 f2). The reference calls that mix from one Python thread per simulated device
// (TF2 CIFAR100_dataset/federated_learning_keras_consensus_FL_threads_CIFAR100.py:674-681, mixing
// at MNIST_dataset/consensus/consensus_v3.py:144-157), so the pool is entered concurrently.
//
// Protocol (one run at a time; a caller that finds the pool busy copies on its own thread):
//   - run() owns the job list for the run (copied into pool storage), resets the claim counter
//     and the completion count, then publishes ONE atomic word  state = gen << 8 | helpers.
//   - A worker takes its part in a run from a single load of that word: worker `id` helps
//     generation g exactly when it observes g and id < helpers(g). The generation and the helper
//     count can never come from two different runs.
//   - A helper of generation g is counted in pending(g), so run g cannot return (and run g + 1
//     cannot start) until that helper has finished with the job list. A worker therefore only
//     ever skips generations that did not need it, and never touches the job list of a run it
//     did not claim.
//   - run()'s wait is bounded: past `timeout` the pool is marked broken, run() returns false so
//     the caller can fail with a message instead of spinning forever, and every later run copies
//     on its caller's thread, so the pool's job list and counters are left to the stragglers.
// Workers spin for ~50 us after each run before parking on a condition variable, so the runs of
// one pipelined call (one per chunk, tens of microseconds apart) do not pay a futex wake-up each.
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

  // Stops and joins the workers. Only for pools that are not broken (a broken pool may have a
  // worker stuck in a copy; the library's process-wide pool is never destroyed).
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
  // the helpers did not finish within `timeout` (the pool is then broken; see above).
  bool run(const Copy* jobs, size_t njobs, int threads,
           std::chrono::nanoseconds timeout = std::chrono::seconds(30)) {
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
    pending_.store(helpers, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);  // under the lock: a parking worker cannot miss it
      publish(helpers);                    // release: jobs_, next_, pending_ happen-before
    }
    cv_.notify_all();
    drain(jobs_);
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0; pending_.load(std::memory_order_acquire) != 0; ++spin) {
      if (spin < 4096) {
        cpu_relax();
        continue;
      }
      std::this_thread::yield();
      if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > timeout) {
        // stragglers may still read jobs_ and bump next_ / pending_: a broken pool never touches
        // them again (every later run copies on its caller's thread)
        broken_.store(true, std::memory_order_relaxed);
        return false;
      }
    }
    return true;
  }

  bool broken() const { return broken_.load(std::memory_order_relaxed); }
  int workers() const { return int(workers_.size()); }
  uint64_t generation() const { return state_.load(std::memory_order_relaxed) >> 8; }

 private:
  // Caller holds mu_. Bumps the generation and sets the helper count in one store.
  void publish(int helpers) {
    const uint64_t gen = (state_.load(std::memory_order_relaxed) >> 8) + 1;
    state_.store(gen << 8 | uint64_t(helpers), std::memory_order_release);
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
         i = next_.fetch_add(1, std::memory_order_relaxed))
      std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
  }

  // One load of state_ that differs from `seen`'s generation: spin, then park.
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
      else std::this_thread::yield();  // oversubscribed: give the core to the caller
    }
  }

  void loop(int id, uint64_t seen) {
    for (;;) {
      const uint64_t s = await(seen);
      seen = s >> 8;
      if (stop_.load(std::memory_order_relaxed)) return;
      if (id >= int(s & 0xff)) continue;  // not a helper of generation `seen`
      drain(jobs_);  // stable until pending_ reaches zero
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
  std::vector<Copy> jobs_;  // the current run's job list (pool-owned: outlives the caller's)
  std::atomic<size_t> next_{0};
  std::atomic<int> pending_{0};
  std::atomic<uint64_t> state_{0};  // gen << 8 | helpers
  std::atomic<bool> stop_{false}, broken_{false};
};

}  // namespace cfa

#endif  // CFA_COPYPOOL_H
