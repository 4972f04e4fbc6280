// hostmix_stress.cpp — the product's drop-in host pipeline (federated_amd/csrc/cfa_hostmix.cpp,
// cfa_host_mix_f32) run on the CPU against the HIP/kernel emulation of tests/native/hostmix_stub:
// several caller threads at once (the reference's one thread per device, TF2
// CIFAR100_dataset/...FL_threads_CIFAR100.py:674-681), random layer layouts (empty layers
// included), fan-ins 0..9, chunk sizes from 4 elements up, 1..8 copy threads, with and without
// divisors, on their own streams or the shared default stream. Every output must equal the
// sequential rule evaluated directly, bit for bit. Built plainly and under ThreadSanitizer by
// tests/test_hostmix_native.py.
//
// usage: hostmix_stress CALLERS ITERS SEED
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "cfa_engine.h"
#include "hip/hip_runtime_api.h"

extern "C" {
hipStream_t stub_stream_create();
void stub_stream_destroy(hipStream_t s);
long stub_launches();
const char* stub_last_error();
}

namespace {
std::atomic<int> failures{0};

void caller(int id, int iters, unsigned long long seed) {
  std::mt19937_64 rng(seed * 7919 + id);
  hipStream_t st = (id % 2) ? stub_stream_create() : nullptr;
  std::vector<float> staging, out_pinned;
  for (int it = 0; it < iters && failures.load() == 0; ++it) {
    const int L = 1 + int(rng() % 6);
    const int n = int(rng() % 10);
    std::vector<size_t> sizes(static_cast<size_t>(L));
    for (auto& s : sizes) s = (rng() % 7 == 0) ? 0 : size_t(rng() % 30000);
    size_t P = 0;
    for (size_t s : sizes) P += s;
    std::normal_distribution<float> nd;
    std::vector<std::vector<std::vector<float>>> in(size_t(n + 1), std::vector<std::vector<float>>(size_t(L)));
    std::vector<const float*> in_ptrs(size_t(n + 1) * L);
    for (int m = 0; m <= n; ++m)
      for (int k = 0; k < L; ++k) {
        auto& v = in[size_t(m)][size_t(k)];
        v.resize(sizes[size_t(k)] + 1);  // non-null even when empty
        for (auto& x : v) x = nd(rng);
        in_ptrs[size_t(m) * L + k] = v.data();
      }
    std::vector<std::vector<float>> out(static_cast<size_t>(L));
    std::vector<float*> out_ptrs(static_cast<size_t>(L));
    for (int k = 0; k < L; ++k) {
      out[size_t(k)].assign(sizes[size_t(k)] + 1, -7.0f);
      out_ptrs[size_t(k)] = out[size_t(k)].data();
    }
    std::vector<float> alphas(static_cast<size_t>(n)), divisors(static_cast<size_t>(n));
    for (int j = 0; j < n; ++j) {
      alphas[size_t(j)] = 1.0f / float(n + 1) + 0.01f * float(j);
      divisors[size_t(j)] = float(1 + rng() % 9);
    }
    const bool div = rng() % 2;
    const size_t chunk = 4 + size_t(rng() % 20000);
    const int threads = 1 + int(rng() % 8);
    const size_t need = cfa_host_mix_staging_elems(sizes.data(), L, n, chunk);
    staging.assign(need + 16, 0.0f);
    out_pinned.assign(P + 1, 0.0f);
    const int rc = cfa_host_mix_f32(out_ptrs.data(), in_ptrs.data(), sizes.data(), L, n, n ? alphas.data() : nullptr,
                                    div && n ? divisors.data() : nullptr, staging.data(), staging.size(),
                                    out_pinned.data(), chunk, threads, st);
    if (rc != CFA_OK) {
      std::fprintf(stderr, "caller %d iter %d: rc %d (%s)\n", id, it, rc, stub_last_error());
      failures.fetch_add(1);
      break;
    }
    for (int k = 0; k < L && failures.load() == 0; ++k) {
      for (size_t i = 0; i < sizes[size_t(k)]; ++i) {
        float w = in[0][size_t(k)][i];
        for (int j = 0; j < n; ++j) {
          float t = in[size_t(j + 1)][size_t(k)][i] - w;
          t = alphas[size_t(j)] * t;
          if (div) t = t / divisors[size_t(j)];
          w = w + t;
        }
        if (std::memcmp(&w, &out[size_t(k)][i], 4) != 0) {
          std::fprintf(stderr, "caller %d iter %d layer %d elem %zu: %g != %g (L %d n %d chunk %zu threads %d)\n", id,
                       it, k, i, out[size_t(k)][i], w, L, n, chunk, threads);
          failures.fetch_add(1);
          break;
        }
      }
      if (out[size_t(k)][sizes[size_t(k)]] != -7.0f) {
        std::fprintf(stderr, "caller %d iter %d layer %d: wrote past the layer\n", id, it, k);
        failures.fetch_add(1);
      }
    }
  }
  if (st) stub_stream_destroy(st);
}
}  // namespace

int main(int argc, char** argv) {
  const int callers = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  const unsigned long long seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
  std::vector<std::thread> ts;
  for (int c = 0; c < callers; ++c) ts.emplace_back(caller, c, iters, seed);
  for (auto& t : ts) t.join();
  if (failures.load()) {
    std::fprintf(stderr, "%d failures\n", failures.load());
    return 1;
  }
  std::printf("OK %d callers x %d calls, %ld chunk launches\n", callers, iters, stub_launches());
  return 0;
}
