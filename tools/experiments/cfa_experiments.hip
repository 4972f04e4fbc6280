// cfa_experiments.hip — measurement-only kernels, built into lib/libcfa_exp.so by `make exp` for
// tools/ (never loaded by the product, not part of the product build): cache-policy,
// traversal-order and read/write decomposition variants of the 8-neighbour mix, allocations with
// explicit hipExtMalloc flags or the VMM API, the contention stand-in, completion-signal forms and
// the read:write ceiling kernels. Results are recorded under profiles/ (DESIGN.md section 3).
// Variants that were tried and not kept (write batching, one-launch multi-device mix, software-
// pipelined mix, the fp64-reciprocal division before it moved into the product) were removed in
// round 5; their code is in commit 27eae93 and their measurements stay under profiles/.
#include "cfa_internal.h"

extern "C" __attribute__((visibility("default"))) const char* cfa_exp_last_error(void) {
  return g_last_error.c_str();
}

// ------------------------------------------------------------------------------------------
// Experiment (not part of the public header): the N = 8, 4-vector mix through buffer loads /
// stores with explicit gfx950 cache-policy bits (aux: 1 = sc0, 2 = nt, 16 = sc1), used by
// tools/tune_cache_policy.py to pick the streaming policy of the production kernel.
// ------------------------------------------------------------------------------------------
namespace {
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void mix8_buf_kernel(float* out, Fanin f, long long nvec) {
  constexpr int N = 8, U = 4;
  const unsigned bytes = (unsigned)(nvec * 16);
  __amdgpu_buffer_rsrc_t r[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) r[k] = __builtin_amdgcn_make_buffer_rsrc((void*)f.src[k], 0, bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, bytes, 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const int base = (int)((t * kTile + threadIdx.x) * 16);
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        u4 x = __builtin_amdgcn_raw_buffer_load_b128(r[k], base + u * kBlock * 16, 0, LAUX);
        v[u][k] = __builtin_bit_cast(f4, x);
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 y = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w, base + u * kBlock * 16, 0, SAUX);
    }
  }
}
// global nt loads (as the production kernel) + buffer store with explicit policy
template <int SAUX>
__global__ __launch_bounds__(kBlock) void mix8_gld_bst_kernel(float* out, Fanin f, long long nvec) {
  constexpr int N = 8, U = 4;
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<true>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 y = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w,
                                             (int)((base + (long long)u * kBlock) * 16), 0, SAUX);
    }
  }
}
// Traversal-order experiment: 0 = grid-stride (production), 1 = blocked (each workgroup owns a
// contiguous span of tiles), 2 = XCD-grouped grid-stride (blocks are dispatched round-robin over
// the 8 XCDs; the logical id is remapped so each XCD walks a contiguous run of tiles).
// Decomposition: 3 = the 9 reads alone (grid-stride), 4 = the output write alone.
template <int MODE>
__global__ __launch_bounds__(kBlock) void mix8_trav_kernel(float* out, Fanin f, long long nvec) {
  constexpr int N = 8, U = 4;
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  const long long G = gridDim.x;
  long long t0, t1, step;
  if constexpr (MODE == 1) {
    t0 = full * blockIdx.x / G;
    t1 = full * (blockIdx.x + 1) / G;
    step = 1;
  } else if constexpr (MODE == 2) {
    const long long per = G / 8;  // host guarantees G % 8 == 0
    t0 = (blockIdx.x % 8) * per + blockIdx.x / 8;
    t1 = full;
    step = G;
  } else {
    t0 = blockIdx.x;
    t1 = full;
    step = G;
  }
  for (long long t = t0; t < t1; t += step) {
    const long long base = t * kTile + threadIdx.x;
    if constexpr (MODE == 4) {  // write-only: the output stream alone
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const f4 y = {f.c[1], f.c[2], f.c[3], (float)u};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w,
                                               (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
      }
      continue;
    }
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<true>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 y = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      if constexpr (MODE == 3) {  // read-only: a store that never fires keeps the loads live
        if (y.x == 1234.5f && y.y == -1234.5f)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w,
                                                 (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w,
                                               (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
      }
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_buf(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P,
    int laux, int saux, int blocks_per_cu, void* stream) {
  if (P % 4096 || P * 4 > 0xffffffffull) return fail(CFA_E_INVALID, "experiment needs P %% 4096 == 0, < 4 GiB");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 8; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  const unsigned grid = grid_for(nvec / (kBlock * 4), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_X(L, S) \
  if (laux == L && saux == S) { mix8_buf_kernel<L, S><<<grid, kBlock, 0, st>>>(out, f, nvec); return check_launch("mix8_buf"); }
  CFA_X(0, 0) CFA_X(2, 2) CFA_X(2, 0) CFA_X(0, 2) CFA_X(1, 2) CFA_X(16, 2) CFA_X(17, 2) CFA_X(3, 2)
  CFA_X(18, 2) CFA_X(19, 2) CFA_X(2, 16) CFA_X(2, 17) CFA_X(2, 18) CFA_X(2, 19) CFA_X(18, 18) CFA_X(17, 17)
  CFA_X(16, 16) CFA_X(1, 1)
#undef CFA_X
#define CFA_G(S) \
  if (laux == -2 && saux == S) { mix8_gld_bst_kernel<S><<<grid, kBlock, 0, st>>>(out, f, nvec); return check_launch("mix8_gld"); }
  CFA_G(0) CFA_G(2) CFA_G(16) CFA_G(17) CFA_G(18) CFA_G(1)
#undef CFA_G
  return fail(CFA_E_INVALID, "policy pair not instantiated");
}

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_traverse(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P,
    int mode, int blocks_per_cu, void* stream) {
  if (P % 4096 || P * 4 > 0xffffffffull) return fail(CFA_E_INVALID, "experiment needs P %% 4096 == 0, < 4 GiB");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 8; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  unsigned grid = grid_for(nvec / (kBlock * 4), lc);
  if (mode == 2) grid -= grid % 8;  // modes 3/4: grid-stride like 0
  if (grid == 0) return fail(CFA_E_INVALID, "experiment grid too small");
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0) mix8_trav_kernel<0><<<grid, kBlock, 0, st>>>(out, f, nvec);
  else if (mode == 1) mix8_trav_kernel<1><<<grid, kBlock, 0, st>>>(out, f, nvec);
  else if (mode == 2) mix8_trav_kernel<2><<<grid, kBlock, 0, st>>>(out, f, nvec);
  else if (mode == 3) mix8_trav_kernel<3><<<grid, kBlock, 0, st>>>(out, f, nvec);
  else if (mode == 4) mix8_trav_kernel<4><<<grid, kBlock, 0, st>>>(out, f, nvec);
  else return fail(CFA_E_INVALID, "unknown traversal mode");
  return check_launch("mix8_trav");
}

// Experiment (not part of the public header): device allocations with explicit hipExtMalloc
// flags (0 default, 3 uncached, 4 physically contiguous), for tools/alloc_experiment.py.
extern "C" __attribute__((visibility("default"))) int cfa_experimental_malloc(void** p, size_t bytes,
                                                                              unsigned flags) {
  hipError_t e = hipExtMallocWithFlags(p, bytes, flags);
  if (e != hipSuccess) return fail(CFA_E_HIP, "hipExtMallocWithFlags(%zu, 0x%x): %s", bytes, flags, hipGetErrorString(e));
  return CFA_OK;
}
extern "C" __attribute__((visibility("default"))) int cfa_experimental_free(void* p) {
  hipError_t e = hipFree(p);
  if (e != hipSuccess) return fail(CFA_E_HIP, "hipFree: %s", hipGetErrorString(e));
  return CFA_OK;
}

// Experiment (not part of the public header): a device buffer through the virtual-memory API, for
// tools/probe/vmm_placement.py: one reserved VA range backed by physical handles of `chunk` bytes
// each (rounded up to the allocation granularity; 0 = one handle for the whole range), mapped in
// order and made read-write for `device`. Freed with cfa_experimental_vmm_free(ptr, bytes, chunk).
namespace {
hipMemAllocationProp vmm_prop(int device) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  return prop;
}
size_t vmm_round(size_t x, size_t g) { return (x + g - 1) / g * g; }
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_vmm_granularity(int device, size_t* min_g,
                                                                                       size_t* rec_g) {
  hipMemAllocationProp prop = vmm_prop(device);
  CFA_HIP_CHECK(hipMemGetAllocationGranularity(min_g, &prop, hipMemAllocationGranularityMinimum));
  CFA_HIP_CHECK(hipMemGetAllocationGranularity(rec_g, &prop, hipMemAllocationGranularityRecommended));
  return CFA_OK;
}

extern "C" __attribute__((visibility("default"))) int cfa_experimental_vmm_alloc(void** p, size_t bytes, size_t chunk,
                                                                                 int device) {
  if (!p || !bytes) return fail(CFA_E_INVALID, "vmm: bad arguments");
  hipMemAllocationProp prop = vmm_prop(device);
  size_t g = 0;
  CFA_HIP_CHECK(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
  const size_t total = vmm_round(bytes, g);
  const size_t step = chunk ? std::min(total, vmm_round(chunk, g)) : total;
  void* base = nullptr;
  CFA_HIP_CHECK(hipMemAddressReserve(&base, total, std::max<size_t>(g, size_t(1) << 30), nullptr, 0));
  for (size_t off = 0; off < total; off += step) {
    const size_t n = std::min(step, total - off);
    hipMemGenericAllocationHandle_t h;
    hipError_t e = hipMemCreate(&h, n, &prop, 0);
    if (e == hipSuccess) {
      e = hipMemMap(static_cast<char*>(base) + off, n, 0, h, 0);
      (void)hipMemRelease(h);  // the mapping keeps the physical memory alive
    }
    if (e != hipSuccess) return fail(CFA_E_HIP, "vmm: create/map at %zu of %zu: %s", off, total, hipGetErrorString(e));
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CFA_HIP_CHECK(hipMemSetAccess(base, total, &acc, 1));
  *p = base;
  return CFA_OK;
}

extern "C" __attribute__((visibility("default"))) int cfa_experimental_vmm_free(void* p, size_t bytes, size_t chunk,
                                                                                int device) {
  hipMemAllocationProp prop = vmm_prop(device);
  size_t g = 0;
  CFA_HIP_CHECK(hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended));
  const size_t total = vmm_round(bytes, g);
  const size_t step = chunk ? std::min(total, vmm_round(chunk, g)) : total;
  for (size_t off = 0; off < total; off += step)
    CFA_HIP_CHECK(hipMemUnmap(static_cast<char*>(p) + off, std::min(step, total - off)));
  CFA_HIP_CHECK(hipMemAddressFree(p, total));
  return CFA_OK;
}


// ------------------------------------------------------------------------------------------
// Contention experiment (tools/probe/contention.py): how much do the mixes of a round slow down
// while another kernel holds a few CUs (as RCCL's copy kernels do during a halo exchange), and
// does handing tiles out dynamically (one device-scope counter, the next tile fetched while the
// current one streams) recover it? `hog`: `blocks` workgroups copy n float4 `reps` times
// (bounded work). `mix8_dyn`: the production mix (nt loads, sc1 buffer stores) with dynamic
// tiles; the counter is zeroed by the host before each launch.
// ------------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(kBlock) void hog_kernel(f4* dst, const f4* src, long long n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += (long long)gridDim.x * kBlock)
      dst[i] = src[i] + (float)r;
}

__global__ __launch_bounds__(kBlock) void mix8_dyn_kernel(float* out, Fanin f, long long nvec,
                                                         unsigned long long* counter) {
  constexpr int N = 8, U = 4;
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  __shared__ long long slot[2];
  if (threadIdx.x == 0) slot[0] = (long long)atomicAdd(counter, 1ull);
  __syncthreads();
  long long t = slot[0];
  int p = 0;
  while (t < full) {
    if (threadIdx.x == 0) slot[p ^ 1] = (long long)atomicAdd(counter, 1ull);  // next tile, in flight
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<true>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 y = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), w,
                                             (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
    }
    __syncthreads();
    p ^= 1;
    t = slot[p];
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_hog(float* dst, const float* src, size_t n,
                                                                           int blocks, int reps, void* stream) {
  if (n % 4 || blocks < 1 || reps < 1) return fail(CFA_E_INVALID, "hog: n %% 4, blocks, reps");
  hog_kernel<<<blocks, kBlock, 0, (hipStream_t)stream>>>((f4*)dst, (const f4*)src, (long long)n / 4, reps);
  return check_launch("hog");
}

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_dyn(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P,
    unsigned long long* counter, int blocks_per_cu, void* stream) {
  if (P % 4096 || P * 4 > 0xffffffffull) return fail(CFA_E_INVALID, "experiment needs P %% 4096 == 0, < 4 GiB");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 8; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  const unsigned grid = grid_for(nvec / (kBlock * 4), lc);
  hipStream_t st = (hipStream_t)stream;
  CFA_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(*counter), st));
  mix8_dyn_kernel<<<grid, kBlock, 0, st>>>(out, f, nvec, counter);
  return check_launch("mix8_dyn");
}

// ------------------------------------------------------------------------------------------
// Standalone compression epilogue variants (tools/probe/compress_sweep.py): U float4 of y and
// ref per lane, nontemporal or default loads / stores, workgroups per CU.
// ------------------------------------------------------------------------------------------
namespace {
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void compress_x_kernel(float* y, const float* ref, long long nvec,
                                                           CompressParams cp) {
  unsigned kept = 0;
  constexpr long long kTile = (long long)kBlock * U;
  for (long long base = (long long)blockIdx.x * kTile + threadIdx.x; base < nvec;
       base += (long long)gridDim.x * kTile) {
    f4 v[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      v[u] = i < nvec ? ld4<NTL>(y, i) : f4{0.f, 0.f, 0.f, 0.f};
      r[u] = i < nvec ? ld4<NTL>(ref, i) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      if (i >= nvec) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = compress_one(v[u][c], r[u][c], cp, kept);
      st4<NTS>(y, i, v[u]);
    }
  }
  block_add_count(kept, cp.kept);
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_compress(
    float* y, const float* ref, size_t P, int mode, unsigned long long* kept, int u, int ntl, int nts,
    int blocks_per_cu, void* stream) {
  if (P % 4 || !y || !ref || !kept) return fail(CFA_E_INVALID, "compress experiment: P %% 4, null buffers");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  cp.cbegin = 0;
  cp.cend = (long long)P;
  cp.kept = kept;
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  const unsigned grid = grid_for((nvec + kBlock * u - 1) / (kBlock * u), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_C(U, L, S) \
  if (u == U && ntl == L && nts == S) { compress_x_kernel<U, L, S><<<grid, kBlock, 0, st>>>(y, ref, nvec, cp); return check_launch("compress_x"); }
  CFA_C(1, 1, 1) CFA_C(2, 1, 1) CFA_C(4, 1, 1) CFA_C(8, 1, 1)
  CFA_C(4, 1, 0) CFA_C(4, 0, 1) CFA_C(4, 0, 0) CFA_C(2, 1, 0) CFA_C(8, 1, 0)
#undef CFA_C
  return fail(CFA_E_INVALID, "variant not instantiated");
}

// ------------------------------------------------------------------------------------------
// Completion-signal experiment (tools/probe/flag_sync.py): a small zero-copy drop-in call is
// launch + kernel + hipStreamSynchronize, and the wake-up of the blocking synchronisation is a
// large part of its round trip. Here the completion is a sequence number written into a pinned
// host word after the mix, and the host spins on that word:
//   method 0: hipStreamWriteValue32 on the stream after the mix;
//   method 1: a one-lane kernel after the mix stores the word (system-scope release);
//   fused:    the mix kernel itself: every workgroup releases its stores at system scope and
//             counts itself in a device counter; the last one resets the counter and stores the
//             word (cfa_experimental_mix2_flag, n = 2, the C1 shape).
// ------------------------------------------------------------------------------------------
namespace {
__global__ void flag_kernel(unsigned* flag, unsigned seq) {
  __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(kBlock) void mix2_flag_kernel(float* out, Fanin f, long long nvec,
                                                           unsigned* counter, unsigned* flag,
                                                           unsigned seq) {
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec;
       i += (long long)gridDim.x * kBlock) {
    f4 v[3];
#pragma unroll
    for (int k = 0; k <= 2; ++k) v[k] = ld4<false>(f.src[k], i);
    st4<false>(out, i, fold<2, CFA_RULE_SEQUENTIAL>(v, f));
  }
  // each wave waits for its own stores (system-scope release), then the workgroup counts itself
  __atomic_thread_fence(__ATOMIC_RELEASE);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_signal(void* stream, unsigned* flag_dev,
                                                                              unsigned seq, int method) {
  hipStream_t st = (hipStream_t)stream;
  if (method == 0) {
    CFA_HIP_CHECK(hipStreamWriteValue32(st, flag_dev, seq, 0));
    return CFA_OK;
  }
  flag_kernel<<<1, 1, 0, st>>>(flag_dev, seq);
  return check_launch("flag_kernel");
}

// Spins until *flag == seq (acquire) or max_spins polls pass; 0 = seen, 1 = timed out.
extern "C" __attribute__((visibility("default"))) int cfa_experimental_wait_flag(const unsigned* flag, unsigned seq,
                                                                                 long long max_spins) {
  for (long long i = 0; i < max_spins; ++i) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return 0;
    __builtin_ia32_pause();
  }
  return 1;
}

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix2_flag(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P,
    unsigned* counter_dev, unsigned* flag_dev, unsigned seq, void* stream) {
  if (P % 4 || !out || !local || !nbrs) return fail(CFA_E_INVALID, "mix2_flag: P %% 4, null buffers");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 2; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  const unsigned grid = (unsigned)std::min<long long>((nvec + kBlock - 1) / kBlock, 1024);
  mix2_flag_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>(out, f, nvec, counter_dev, flag_dev, seq);
  return check_launch("mix2_flag");
}

// ------------------------------------------------------------------------------------------
// Cache-policy experiment at the round-2 launch shape (tools/probe/policy_shape.py): round 1 chose
// the streaming policy (nt loads, sc1 store) with 4 float4 per lane and two workgroups per CU;
// the production default is now one workgroup per CU with 2 float4 per lane. The N = 8 mix through
// buffer loads / stores with explicit policy bits (aux: 1 = sc0, 2 = nt, 16 = sc1), U float4 per
// lane, same fold: the output is identical to production.
// ------------------------------------------------------------------------------------------
namespace {
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void mix8_pol_kernel(float* out, Fanin f, long long nvec) {
  constexpr int N = 8;
  const unsigned bytes = (unsigned)(nvec * 16);
  __amdgpu_buffer_rsrc_t r[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) r[k] = __builtin_amdgcn_make_buffer_rsrc((void*)f.src[k], 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, bytes, 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const int base = (int)((t * kTile + threadIdx.x) * 16);
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u][k] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r[k], base + u * kBlock * 16, 0, LAUX));
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, fold<N, CFA_RULE_SEQUENTIAL>(v[u], f)), w,
                                             base + u * kBlock * 16, 0, SAUX);
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      f4 v[N + 1];
#pragma unroll
      for (int k = 0; k <= N; ++k) v[k] = ld4<false>(f.src[k], i);
      st4<false>(out, i, fold<N, CFA_RULE_SEQUENTIAL>(v, f));
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_policy(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P, int u, int laux,
    int saux, int blocks_per_cu, void* stream) {
  if (P % 4 || P * 4 > 0x7ffffff0ull) return fail(CFA_E_INVALID, "policy experiment: P %% 4, P * 4 < 2 GiB");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 8; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  const unsigned grid = grid_for(nvec / (kBlock * u), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_Q(U, L, S) \
  if (u == U && laux == L && saux == S) { mix8_pol_kernel<U, L, S><<<grid, kBlock, 0, st>>>(out, f, nvec); return check_launch("mix8_pol"); }
  CFA_Q(2, 2, 16) CFA_Q(2, 0, 16) CFA_Q(2, 16, 16) CFA_Q(2, 17, 16) CFA_Q(2, 18, 16) CFA_Q(2, 3, 16)
  CFA_Q(2, 1, 16) CFA_Q(2, 2, 2) CFA_Q(2, 2, 0) CFA_Q(2, 2, 17) CFA_Q(2, 2, 18) CFA_Q(2, 2, 1)
  CFA_Q(1, 2, 16) CFA_Q(4, 2, 16)
#undef CFA_Q
  return fail(CFA_E_INVALID, "policy variant not instantiated");
}

// ------------------------------------------------------------------------------------------
// Store-form experiment (tools/probe/store_form.py): production loads (global, nt) with the output
// stored as 0 = buffer store sc1 (production), 1 = global store nt, 2 = buffer store nt,
// 3 = global store sc1, 4 = global store nt sc1 (3 and 4 as inline vector-store asm: no builtin
// names those bits on a global store). U float4 per lane; identical output.
// ------------------------------------------------------------------------------------------
namespace {
template <int U, int MODE>
__global__ __launch_bounds__(kBlock) void mix8_store_kernel(float* out, Fanin f, long long nvec) {
  constexpr int N = 8;
  const __amdgpu_buffer_rsrc_t w =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<true>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 y = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      const long long i = base + (long long)u * kBlock;
      if constexpr (MODE == 0)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y), w, (int)(i * 16), 0, kStoreSc1);
      else if constexpr (MODE == 1)
        __builtin_nontemporal_store(y, reinterpret_cast<f4*>(out) + i);
      else if constexpr (MODE == 2)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y), w, (int)(i * 16), 0, 2);
      else if constexpr (MODE == 3)
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(reinterpret_cast<f4*>(out) + i), "v"(y) : "memory");
      else
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(reinterpret_cast<f4*>(out) + i), "v"(y) : "memory");
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      f4 v[N + 1];
#pragma unroll
      for (int k = 0; k <= N; ++k) v[k] = ld4<false>(f.src[k], i);
      st4<false>(out, i, fold<N, CFA_RULE_SEQUENTIAL>(v, f));
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_store(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P, int u, int mode,
    int blocks_per_cu, void* stream) {
  if (P % 4 || P * 4 > 0x7ffffff0ull) return fail(CFA_E_INVALID, "store experiment: P %% 4, P * 4 < 2 GiB");
  Fanin f{};
  f.src[0] = local;
  for (int j = 0; j < 8; ++j) {
    f.src[j + 1] = nbrs[j];
    f.c[j + 1] = alphas[j];
  }
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{blocks_per_cu, 4, 0};
  const unsigned grid = grid_for(nvec / (kBlock * u), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_S(U, M) \
  if (u == U && mode == M) { mix8_store_kernel<U, M><<<grid, kBlock, 0, st>>>(out, f, nvec); return check_launch("mix8_store"); }
  CFA_S(2, 0) CFA_S(2, 1) CFA_S(2, 2) CFA_S(2, 3) CFA_S(2, 4) CFA_S(1, 1) CFA_S(4, 1)
#undef CFA_S
  return fail(CFA_E_INVALID, "store variant not instantiated");
}

// Graph-replayable completion signal (tools/probe/flag_sync.py, graph variant): a device counter
// is bumped and its new value stored into the pinned host word, so the same captured kernel
// signals a fresh value at every replay (the host expects previous + 1).
namespace {
__global__ void flag_inc_kernel(unsigned* counter_dev, unsigned* flag) {
  const unsigned v = __hip_atomic_fetch_add(counter_dev, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace
extern "C" __attribute__((visibility("default"))) int cfa_experimental_signal_inc(void* stream, unsigned* counter_dev,
                                                                                  unsigned* flag_dev) {
  flag_inc_kernel<<<1, 1, 0, (hipStream_t)stream>>>(counter_dev, flag_dev);
  return check_launch("flag_inc_kernel");
}

// ------------------------------------------------------------------------------------------
// Round 4, the lowest roofline rows (tools/probe/lowrow_sweep.py): the fp64 divisor fold
// (cfa_fold_f64, rule 2), the all-fp64 MEWMA (cfa_mewma_tf1_f64) and the standalone compression
// epilogue (cfa_compress_epilogue_f32) rebuilt on the headline mix's skeleton: full tiles of
// kBlock x U 16-byte vectors per stream walked grid-stride with no per-vector guards (the
// partial tail handled apart by one workgroup), every load of a tile issued before its first use,
// and a chosen store policy (SP: 0 plain global store, 1 nontemporal global store, 2 buffer store
// nt, 3 buffer store sc1). The arithmetic is the production kernels' own, so the output must be
// identical (the sweep checks it bit for bit).
// ------------------------------------------------------------------------------------------
namespace {
typedef double xd2 __attribute__((ext_vector_type(2)));
struct XF64Fanin {
  const double* src[CFA_MAX_FANIN + 1];
  double a[CFA_MAX_FANIN + 1], d[CFA_MAX_FANIN + 1], r[CFA_MAX_FANIN + 1];
  int fast_div;
};
__device__ __forceinline__ double x_ddiv_rn(double a, double b, double rb, bool fast) {
  const double aa = __builtin_fabs(a);
  if (fast && aa >= 0x1p-900 && aa <= 0x1p900) {
    const double q = a * rb;
    const double r = __builtin_fma(-q, b, a);
    return __builtin_fma(r, rb, q);
  }
  return a / b;
}
template <typename V, int SP>
__device__ __forceinline__ void x_store(V* base, __amdgpu_buffer_rsrc_t w, long long i, V v) {
  if constexpr (SP == 0) base[i] = v;
  else if constexpr (SP == 1) __builtin_nontemporal_store(v, base + i);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), w, (int)(i * 16), 0,
                                              SP == 2 ? kStoreNt : kStoreSc1);
}
template <bool NT, typename V>
__device__ __forceinline__ V x_load(const V* p, long long i) {
  if constexpr (NT) return __builtin_nontemporal_load(p + i);
  else return p[i];
}

template <int N>
__device__ __forceinline__ xd2 x_fold_div(const xd2 (&v)[N + 1], const XF64Fanin& f) {
  xd2 y;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    double w = v[0][c];
#pragma unroll
    for (int k = 1; k <= N; ++k) w = w + x_ddiv_rn(f.a[k] * (v[k][c] - w), f.d[k], f.r[k], f.fast_div);
    y[c] = w;
  }
  return y;
}

template <int N, int U, int SP>
__global__ __launch_bounds__(kBlock) void fold64_x_kernel(double* out, XF64Fanin f, long long nvec2) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec2 / kTile;
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec2 * 16), 0x00020000);
  xd2* o = reinterpret_cast<xd2*>(out);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    xd2 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = x_load<true>(reinterpret_cast<const xd2*>(f.src[k]), base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) x_store<xd2, SP>(o, w, base + (long long)u * kBlock, x_fold_div<N>(v[u], f));
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec2; i += kBlock) {
      xd2 v[N + 1];
#pragma unroll
      for (int k = 0; k <= N; ++k) v[k] = reinterpret_cast<const xd2*>(f.src[k])[i];
      o[i] = x_fold_div<N>(v, f);
    }
  }
}

// all-fp64 MEWMA (mask 0), not the initial round: s_j = rho*g_j + (1-rho)*s_j; W -= lr*(filtered ? s_j : g_j)
struct XMewma {
  double* W;
  double* s[4];
  const double* g[4];
  double rho, one_minus_rho, lr1, lr2;
  long long split;  // in elements
  int filtered;
};
template <int N>
__device__ __forceinline__ void x_mewma(xd2& Wv, const xd2 (&g)[N], xd2 (&s)[N], long long e0, const XMewma& a) {
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    double W = Wv[c];
    const double lr = e0 + c < a.split ? a.lr1 : a.lr2;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double sv = a.rho * g[j][c] + a.one_minus_rho * s[j][c];
      s[j][c] = sv;
      W = W - lr * (a.filtered ? sv : g[j][c]);
    }
    Wv[c] = W;
  }
}
template <int N, int U, int SP, bool NTL>
__global__ __launch_bounds__(kBlock) void mewma64_x_kernel(XMewma a, long long nvec2) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec2 / kTile;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, (unsigned)(nvec2 * 16), 0x00020000);
  __amdgpu_buffer_rsrc_t sr[N];
#pragma unroll
  for (int j = 0; j < N; ++j) sr[j] = __builtin_amdgcn_make_buffer_rsrc((void*)a.s[j], 0, (unsigned)(nvec2 * 16), 0x00020000);
  xd2* W2 = reinterpret_cast<xd2*>(a.W);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    xd2 Wv[U], g[U][N], s[U][N];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      Wv[u] = x_load<NTL>(reinterpret_cast<const xd2*>(a.W), i);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        g[u][j] = x_load<true>(reinterpret_cast<const xd2*>(a.g[j]), i);
        s[u][j] = x_load<NTL>(reinterpret_cast<const xd2*>(a.s[j]), i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      x_mewma<N>(Wv[u], g[u], s[u], 2 * i, a);
#pragma unroll
      for (int j = 0; j < N; ++j) x_store<xd2, SP>(reinterpret_cast<xd2*>(a.s[j]), sr[j], i, s[u][j]);
      x_store<xd2, SP>(W2, wr, i, Wv[u]);
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec2; i += kBlock) {
      xd2 Wv = W2[i], g[N], s[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        g[j] = reinterpret_cast<const xd2*>(a.g[j])[i];
        s[j] = reinterpret_cast<const xd2*>(a.s[j])[i];
      }
      x_mewma<N>(Wv, g, s, 2 * i, a);
#pragma unroll
      for (int j = 0; j < N; ++j) reinterpret_cast<xd2*>(a.s[j])[i] = s[j];
      W2[i] = Wv;
    }
  }
}

// Stream-major form of mewma64_x_kernel: every stream's U vectors are loaded back to back (as
// rw_kernel does), and stored the same way, instead of one vector of each stream in turn.
template <int N, int U, int SP, bool NTL>
__global__ __launch_bounds__(kBlock) void mewma64_sm_kernel(XMewma a, long long nvec2) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec2 / kTile;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, (unsigned)(nvec2 * 16), 0x00020000);
  __amdgpu_buffer_rsrc_t sr[N];
#pragma unroll
  for (int j = 0; j < N; ++j) sr[j] = __builtin_amdgcn_make_buffer_rsrc((void*)a.s[j], 0, (unsigned)(nvec2 * 16), 0x00020000);
  xd2* W2 = reinterpret_cast<xd2*>(a.W);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    xd2 Wv[U], g[U][N], s[U][N];
#pragma unroll
    for (int u = 0; u < U; ++u) Wv[u] = x_load<NTL>(reinterpret_cast<const xd2*>(a.W), base + (long long)u * kBlock);
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) g[u][j] = x_load<true>(reinterpret_cast<const xd2*>(a.g[j]), base + (long long)u * kBlock);
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) s[u][j] = x_load<NTL>(reinterpret_cast<const xd2*>(a.s[j]), base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) x_mewma<N>(Wv[u], g[u], s[u], 2 * (base + (long long)u * kBlock), a);
#pragma unroll
    for (int j = 0; j < N; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) x_store<xd2, SP>(reinterpret_cast<xd2*>(a.s[j]), sr[j], base + (long long)u * kBlock, s[u][j]);
#pragma unroll
    for (int u = 0; u < U; ++u) x_store<xd2, SP>(W2, wr, base + (long long)u * kBlock, Wv[u]);
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec2; i += kBlock) {
      xd2 Wv = W2[i], g[N], s[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        g[j] = reinterpret_cast<const xd2*>(a.g[j])[i];
        s[j] = reinterpret_cast<const xd2*>(a.s[j])[i];
      }
      x_mewma<N>(Wv, g, s, 2 * i, a);
#pragma unroll
      for (int j = 0; j < N; ++j) reinterpret_cast<xd2*>(a.s[j])[i] = s[j];
      W2[i] = Wv;
    }
  }
}

// Software-pipelined form of mewma64_x_kernel (round 4): the loads of a workgroup's next tile are
// issued BEFORE the current tile is computed and stored. vmcnt counts loads and stores together in
// issue order (MI355X_MICROARCH.md), so in the plain loop the first use of tile t+1's loads also
// waits for every store of tile t; here the stores of tile t are younger than tile t+1's loads
// and the wait leaves them in flight. Two tiles of registers per lane.
template <int N, int U>
struct MewmaTile {
  xd2 W[U], g[U][N], s[U][N];
};
template <int N, int U, bool NTL>
__device__ __forceinline__ void mewma_tile_load(MewmaTile<N, U>& T, const XMewma& a, long long base) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * kBlock;
    T.W[u] = x_load<NTL>(reinterpret_cast<const xd2*>(a.W), i);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      T.g[u][j] = x_load<true>(reinterpret_cast<const xd2*>(a.g[j]), i);
      T.s[u][j] = x_load<NTL>(reinterpret_cast<const xd2*>(a.s[j]), i);
    }
  }
}
template <int N, int U, int SP>
__device__ __forceinline__ void mewma_tile_store(MewmaTile<N, U>& T, const XMewma& a, long long base,
                                                 __amdgpu_buffer_rsrc_t wr, const __amdgpu_buffer_rsrc_t (&sr)[N]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * kBlock;
    x_mewma<N>(T.W[u], T.g[u], T.s[u], 2 * i, a);
#pragma unroll
    for (int j = 0; j < N; ++j) x_store<xd2, SP>(reinterpret_cast<xd2*>(a.s[j]), sr[j], i, T.s[u][j]);
    x_store<xd2, SP>(reinterpret_cast<xd2*>(a.W), wr, i, T.W[u]);
  }
}
template <int N, int U, int SP, bool NTL>
__global__ __launch_bounds__(kBlock) void mewma64_pipe_kernel(XMewma a, long long nvec2) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec2 / kTile;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.W, 0, (unsigned)(nvec2 * 16), 0x00020000);
  __amdgpu_buffer_rsrc_t sr[N];
#pragma unroll
  for (int j = 0; j < N; ++j) sr[j] = __builtin_amdgcn_make_buffer_rsrc((void*)a.s[j], 0, (unsigned)(nvec2 * 16), 0x00020000);
  long long t = blockIdx.x;
  if (t < full) {
    MewmaTile<N, U> A, B;
    mewma_tile_load<N, U, NTL>(A, a, t * kTile + threadIdx.x);
    // two tiles per trip, A and B alternating, so no register copies between the roles. The next
    // tile's loads are unconditional (past the last tile they re-read the current one, whose values
    // are then discarded): a load behind a branch makes the wait after the join a vmcnt(0).
    for (;;) {
      const long long t1 = t + gridDim.x;
      mewma_tile_load<N, U, NTL>(B, a, (t1 < full ? t1 : t) * kTile + threadIdx.x);
      mewma_tile_store<N, U, SP>(A, a, t * kTile + threadIdx.x, wr, sr);
      if (t1 >= full) break;
      const long long t2 = t1 + gridDim.x;
      mewma_tile_load<N, U, NTL>(A, a, (t2 < full ? t2 : t1) * kTile + threadIdx.x);
      mewma_tile_store<N, U, SP>(B, a, t1 * kTile + threadIdx.x, wr, sr);
      if (t2 >= full) break;
      t = t2;
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    xd2* W2 = reinterpret_cast<xd2*>(a.W);
    for (long long i = full * kTile + threadIdx.x; i < nvec2; i += kBlock) {
      xd2 Wv = W2[i], g[N], s[N];
#pragma unroll
      for (int j = 0; j < N; ++j) {
        g[j] = reinterpret_cast<const xd2*>(a.g[j])[i];
        s[j] = reinterpret_cast<const xd2*>(a.s[j])[i];
      }
      x_mewma<N>(Wv, g, s, 2 * i, a);
#pragma unroll
      for (int j = 0; j < N; ++j) reinterpret_cast<xd2*>(a.s[j])[i] = s[j];
      W2[i] = Wv;
    }
  }
}

template <int U, int SP, bool NTL>
__global__ __launch_bounds__(kBlock) void compress_full_kernel(float* y, const float* ref, long long nvec,
                                                              CompressParams cp) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  const __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, (unsigned)(nvec * 16), 0x00020000);
  f4* y4 = reinterpret_cast<f4*>(y);
  unsigned kept = 0;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = x_load<NTL>(reinterpret_cast<const f4*>(y), base + (long long)u * kBlock);
      r[u] = x_load<true>(reinterpret_cast<const f4*>(ref), base + (long long)u * kBlock);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = compress_sel<2>(v[u][c], r[u][c], (float)cp.thr, (float)cp.rep, kept);
      x_store<f4, SP>(y4, w, base + (long long)u * kBlock, v[u]);
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      f4 v = y4[i];
      const f4 r = reinterpret_cast<const f4*>(ref)[i];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = compress_one(v[c], r[c], cp, kept);
      y4[i] = v;
    }
  }
  block_add_count(kept, cp.kept);
}
}  // namespace

// out = fp64 divisor fold of local and n = 4 neighbours (rule 2); u = vectors per stream per lane,
// sp = store policy (above), bpc = workgroups per CU (0: one per tile).
extern "C" __attribute__((visibility("default"))) int cfa_experimental_fold64_div(
    double* out, const double* local, const double* const* nbrs, const double* alphas, const double* divisors,
    size_t P, int u, int sp, int bpc, void* stream) {
  if (P % 2 || P * 8 > 0x7ffffff0ull || ((uintptr_t)out & 15)) return fail(CFA_E_INVALID, "fold64 experiment: P even, < 2 GiB, aligned");
  XF64Fanin f{};
  f.src[0] = local;
  f.fast_div = 1;
  for (int j = 1; j <= 4; ++j) {
    f.src[j] = nbrs[j - 1];
    f.a[j] = alphas[j - 1];
    f.d[j] = divisors[j - 1];
    f.r[j] = 1.0 / f.d[j];
    if (!(f.d[j] >= 0x1p-20 && f.d[j] <= 0x1p20)) f.fast_div = 0;
  }
  const long long nvec2 = (long long)P / 2;
  cfa_launch_t lc{bpc, 4, 0};
  const unsigned grid = grid_for(std::max(1LL, nvec2 / (kBlock * u)), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_F(U, S) \
  if (u == U && sp == S) { fold64_x_kernel<4, U, S><<<grid, kBlock, 0, st>>>(out, f, nvec2); return check_launch("fold64_x"); }
  CFA_F(1, 0) CFA_F(1, 1) CFA_F(1, 2) CFA_F(1, 3) CFA_F(2, 0) CFA_F(2, 1) CFA_F(2, 2) CFA_F(2, 3)
  CFA_F(4, 1) CFA_F(4, 2) CFA_F(1, 3) CFA_F(4, 3)
#undef CFA_F
  return fail(CFA_E_INVALID, "fold64 variant not instantiated");
}

// W, s[0..1] updated in place from g[0..1] (all fp64, not init); ntl = nontemporal loads of W / s.
extern "C" __attribute__((visibility("default"))) int cfa_experimental_mewma64(
    double* W, double* const* s, const double* const* g, double rho, double lr1, double lr2, size_t split,
    int filtered, size_t P, int u, int sp, int ntl, int bpc, void* stream) {
  if (P % 2 || P * 8 > 0x7ffffff0ull) return fail(CFA_E_INVALID, "mewma64 experiment: P even, < 2 GiB");
  XMewma a{};
  a.W = W;
  for (int j = 0; j < 2; ++j) {
    a.s[j] = s[j];
    a.g[j] = g[j];
  }
  a.rho = rho;
  a.one_minus_rho = 1.0 - rho;
  a.lr1 = lr1;
  a.lr2 = lr2;
  a.split = (long long)split;
  a.filtered = filtered;
  const long long nvec2 = (long long)P / 2;
  cfa_launch_t lc{bpc, 4, 0};
  const unsigned grid = grid_for(std::max(1LL, nvec2 / (kBlock * u)), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_M(U, S, L) \
  if (u == U && sp == S && ntl == L) { mewma64_x_kernel<2, U, S, L><<<grid, kBlock, 0, st>>>(a, nvec2); return check_launch("mewma64_x"); }
  CFA_M(1, 1, 1) CFA_M(1, 2, 1) CFA_M(1, 0, 0) CFA_M(2, 1, 1) CFA_M(2, 2, 1) CFA_M(2, 0, 0) CFA_M(1, 3, 1)
  CFA_M(2, 3, 1) CFA_M(1, 3, 0) CFA_M(2, 3, 0) CFA_M(4, 3, 1) CFA_M(4, 1, 1) CFA_M(4, 2, 1)
#undef CFA_M
  // sp + 10: the stream-major load / store order (mewma64_sm_kernel)
#define CFA_SM(U, S, L) \
  if (u == U && sp == S + 10 && ntl == L) { mewma64_sm_kernel<2, U, S, L><<<grid, kBlock, 0, st>>>(a, nvec2); return check_launch("mewma64_sm"); }
  CFA_SM(1, 1, 1) CFA_SM(2, 1, 1) CFA_SM(4, 1, 1) CFA_SM(4, 3, 1) CFA_SM(2, 3, 1) CFA_SM(4, 2, 1)
#undef CFA_SM
  // sp + 20: software-pipelined (mewma64_pipe_kernel)
#define CFA_PI(U, S, L) \
  if (u == U && sp == S + 20 && ntl == L) { mewma64_pipe_kernel<2, U, S, L><<<grid, kBlock, 0, st>>>(a, nvec2); return check_launch("mewma64_pipe"); }
  CFA_PI(1, 1, 1) CFA_PI(2, 1, 1) CFA_PI(1, 3, 1) CFA_PI(2, 3, 1) CFA_PI(1, 2, 1) CFA_PI(2, 2, 1) CFA_PI(4, 3, 1)
  CFA_PI(1, 0, 0) CFA_PI(2, 0, 0)
#undef CFA_PI
  return fail(CFA_E_INVALID, "mewma64 variant not instantiated");
}

// y compressed in place against ref over the whole bucket (P % 4 == 0).
extern "C" __attribute__((visibility("default"))) int cfa_experimental_compress_full(
    float* y, const float* ref, size_t P, int mode, unsigned long long* kept, int u, int sp, int ntl, int bpc,
    void* stream) {
  if (P % 4 || P * 4 > 0x7ffffff0ull || compress_kind(mode) != 2)
    return fail(CFA_E_INVALID, "compress experiment: P %% 4, < 2 GiB, a DPCM mode");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  cp.cbegin = 0;
  cp.cend = (long long)P;
  cp.kept = kept;
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{bpc, 4, 0};
  const unsigned grid = grid_for(std::max(1LL, nvec / (kBlock * u)), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_C(U, S, L) \
  if (u == U && sp == S && ntl == L) { compress_full_kernel<U, S, L><<<grid, kBlock, 0, st>>>(y, ref, nvec, cp); return check_launch("compress_full"); }
  CFA_C(2, 0, 0) CFA_C(4, 0, 0) CFA_C(8, 0, 0) CFA_C(4, 1, 1) CFA_C(4, 2, 1) CFA_C(4, 3, 0) CFA_C(2, 2, 1) CFA_C(4, 1, 0)
#undef CFA_C
  return fail(CFA_E_INVALID, "compress variant not instantiated");
}

// ------------------------------------------------------------------------------------------
// Round 4: read/write-mix ceilings (tools/probe/lowrow_sweep.py --ceilings). R streams read,
// W streams written (dst[w] may alias src[w]: in place), the lightest possible arithmetic
// (dst[w] = src[w] + the sum of all R sources: no load can be dropped), on the same skeleton and store policies as above. The best
// variant's rate is what this hardware streams at that read:write mix, the ceiling a kernel with
// the same mix and no compute can reach.
// ------------------------------------------------------------------------------------------
namespace {
struct RwArgs {
  const float* src[16];
  float* dst[8];
};
template <int R, int W, int U, int SP, bool NTL>
__global__ __launch_bounds__(kBlock) void rw_kernel(RwArgs a, long long nvec) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  __amdgpu_buffer_rsrc_t wr[W];
#pragma unroll
  for (int w = 0; w < W; ++w) wr[w] = __builtin_amdgcn_make_buffer_rsrc((void*)a.dst[w], 0, (unsigned)(nvec * 16), 0x00020000);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][R];
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = x_load<NTL>(reinterpret_cast<const f4*>(a.src[k]), base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 acc = v[u][0];  // every loaded stream feeds every store (no load can be dropped)
#pragma unroll
      for (int k = 1; k < R; ++k) acc = acc + v[u][k];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const f4 y = R > 1 ? acc + v[u][w] : v[u][0];
        x_store<f4, SP>(reinterpret_cast<f4*>(a.dst[w]), wr[w], base + (long long)u * kBlock, y);
      }
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_rw(
    const float* const* src, float* const* dst, int r, int w, size_t P, int u, int sp, int ntl, int bpc, void* stream) {
  if (P % 4 || P * 4 > 0x7ffffff0ull || r < 1 || r > 16 || w < 1 || w > 8)
    return fail(CFA_E_INVALID, "rw experiment: P %% 4, < 2 GiB, 1 <= r <= 16, 1 <= w <= 8");
  RwArgs a{};
  for (int k = 0; k < r; ++k) a.src[k] = src[k];
  for (int k = 0; k < w; ++k) a.dst[k] = dst[k];
  const long long nvec = (long long)P / 4;
  cfa_launch_t lc{bpc, 4, 0};
  const unsigned grid = grid_for(std::max(1LL, nvec / (kBlock * u)), lc);
  hipStream_t st = (hipStream_t)stream;
#define CFA_RW(R, W, U, S, L) \
  if (r == R && w == W && u == U && sp == S && ntl == L) { rw_kernel<R, W, U, S, L><<<grid, kBlock, 0, st>>>(a, nvec); return check_launch("rw"); }
#define CFA_RW_SHAPES(R, W) \
  CFA_RW(R, W, 1, 1, 1) CFA_RW(R, W, 2, 1, 1) CFA_RW(R, W, 4, 1, 1) CFA_RW(R, W, 2, 3, 1) CFA_RW(R, W, 4, 3, 1) \
  CFA_RW(R, W, 2, 2, 1) CFA_RW(R, W, 4, 0, 0) CFA_RW(R, W, 2, 0, 0) CFA_RW(R, W, 4, 3, 0) CFA_RW(R, W, 1, 3, 1)
  CFA_RW_SHAPES(1, 1) CFA_RW_SHAPES(2, 1) CFA_RW_SHAPES(5, 1) CFA_RW_SHAPES(5, 3) CFA_RW_SHAPES(9, 1)
#undef CFA_RW_SHAPES
#undef CFA_RW
  return fail(CFA_E_INVALID, "rw variant not instantiated");
}
