// cfa_mix.hip — the streaming mix kernels (fp32 buckets) and their C-ABI: the sequential CFA rule,
// the FedAvg divisor form, the linear closed form, the fused and standalone compression
// epilogue.
//
// The reference computes the mixing step as numpy AXPY chains over whole tensors, one
// neighbour at a time, with a file round trip between neighbours:
//   TF1/consensus/cfa.py:66-76, cfa_ongraphs.py:109-119, cfa_ge_2stage.py:73-83 / 594-621,
//   TF2 consensus_v3.py:153-155, consensus_v4.py:211-213 / 251-253.
// Here one launch folds every neighbour of a device in registers: each lane streams 16-byte
// slices of the local bucket and of all n neighbour buckets from HBM, applies the rule, and
// writes the result once. The work is HBM-bound (0.2-0.45 flop/byte): no MFMA and no LDS
// staging; coefficients and bucket pointers live in the kernel arguments (SGPRs); every load of
// a tile is issued before its first use; the fan-in N is a template parameter so the fold is
// fully unrolled.
#include <chrono>
#include <thread>

#include "cfa_internal.h"

extern "C" int cfa_version(void) { return CFA_VERSION; }

extern "C" int cfa_host_device_pointer(const void* host, void** dev) {
  if (!host || !dev) return fail(CFA_E_INVALID, "null pointer");
  *dev = nullptr;
  void* p = nullptr;
  hipError_t e = hipHostGetDevicePointer(&p, const_cast<void*>(host), 0);
  if (e != hipSuccess || !p)
    return fail(CFA_E_HIP, "hipHostGetDevicePointer: %s (not pinned host memory?)", hipGetErrorString(e));
  *dev = p;
  return CFA_OK;
}
extern "C" int cfa_device_prepare(int device) {
  int prev = 0;
  CFA_HIP_CHECK(hipGetDevice(&prev));
  if (device != prev) CFA_HIP_CHECK(hipSetDevice(device));
  (void)device_cus();  // fills the shared CU-count cache
  const int rc = grad_prepare_device();
  if (device != prev) CFA_HIP_CHECK(hipSetDevice(prev));
  return rc;
}
extern "C" int cfa_stream_synchronize(void* stream) {
  CFA_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return CFA_OK;
}
extern "C" int cfa_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes && (!dst || !src)) return fail(CFA_E_INVALID, "null copy pointer");
  if (bytes) CFA_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream));
  return CFA_OK;
}
extern "C" int cfa_counter_fetch(unsigned long long* counter, unsigned long long* host_dst, void* stream) {
  if (!counter || !host_dst) return fail(CFA_E_INVALID, "null counter or destination");
  hipStream_t st = (hipStream_t)stream;
  CFA_HIP_CHECK(hipMemcpyAsync(host_dst, counter, sizeof(*counter), hipMemcpyDefault, st));
  CFA_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(*counter), st));
  return CFA_OK;
}
namespace {
// One lane stores the call's value into the caller's pinned host word; stream order puts it after
// every earlier launch of the stream, and the release makes their results visible with it.
__global__ void stream_signal_kernel(unsigned* word, unsigned value) {
  __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace
extern "C" int cfa_stream_signal(unsigned* word_dev, unsigned value, void* stream) {
  if (!word_dev) return fail(CFA_E_INVALID, "null signal word");
  stream_signal_kernel<<<1, 1, 0, (hipStream_t)stream>>>(word_dev, value);
  return check_launch("stream_signal");
}
// The host lane's waits run on the host, never on a stream: a wait parked on the GPU holds every
// stream that shares its hardware queue (4 per process by default), the compute stream included.
// The calling thread polls the pinned word (acquire loads: the producer's release store made its
// copy visible with it) until it reaches `value` in sequence order, spinning for the first
// ~20 us and then sleeping in 20 us steps, and gives up after `timeout_us`; the caller then
// enqueues the copy the word guards. No process-wide state.
extern "C" int cfa_host_wait_word(const unsigned* word_host, unsigned value, long long timeout_us) {
  if (!word_host) return fail(CFA_E_INVALID, "null wait word");
  if (timeout_us <= 0) return fail(CFA_E_INVALID, "timeout_us must be positive (got %lld)", timeout_us);
  auto reached = [&] { return static_cast<int>(__atomic_load_n(word_host, __ATOMIC_ACQUIRE) - value) >= 0; };
  if (reached()) return CFA_OK;
  const auto t0 = std::chrono::steady_clock::now();
  const auto spin = std::chrono::microseconds(20), limit = std::chrono::microseconds(timeout_us);
  for (unsigned i = 1;; ++i) {
    if (reached()) return CFA_OK;
    if ((i & 63) == 0) {
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt > limit) break;
      if (dt > spin) std::this_thread::sleep_for(std::chrono::microseconds(20));
    } else {
      __builtin_ia32_pause();
    }
  }
  if (reached()) return CFA_OK;
  return fail(CFA_E_TIMEOUT, "wait word holds %u after %lld us, expected %u", __atomic_load_n(word_host, __ATOMIC_ACQUIRE),
              timeout_us, value);
}
extern "C" int cfa_host_register(void* host, size_t bytes) {
  if (!host || !bytes) return fail(CFA_E_INVALID, "null or empty host range");
  CFA_HIP_CHECK(hipHostRegister(host, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  return CFA_OK;
}
extern "C" int cfa_host_unregister(void* host) {
  if (!host) return fail(CFA_E_INVALID, "null host pointer");
  CFA_HIP_CHECK(hipHostUnregister(host));
  return CFA_OK;
}
extern "C" int cfa_wait_signal(const unsigned* word_host, unsigned value, void* stream, long long spin_us) {
  if (!word_host) return fail(CFA_E_INVALID, "null signal word");
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    if (__atomic_load_n(word_host, __ATOMIC_ACQUIRE) == value) return CFA_OK;
    __builtin_ia32_pause();
    if ((i & 255) == 255 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us > 0 ? spin_us : 0))
      break;
  }
  CFA_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  if (__atomic_load_n(word_host, __ATOMIC_ACQUIRE) != value)
    return fail(CFA_E_INVALID, "signal word holds %u after the stream completed, expected %u",
                __atomic_load_n(word_host, __ATOMIC_ACQUIRE), value);
  return CFA_OK;
}
extern "C" const char* cfa_last_error(void) { return g_last_error.c_str(); }
// Used by cfa_comm.cpp so every translation unit reports through one thread-local message.
extern "C" __attribute__((visibility("hidden"))) void cfa_internal_set_error(const char* msg) {
  g_last_error = msg ? msg : "";
}

namespace {

// ------------------------------------------------------------------------------------------
// Vector mix kernel: tiles of kBlock*U float4 per block, grid-stride over tiles; the last
// partial tile is handled with per-vector guards by the block that owns it.
// ------------------------------------------------------------------------------------------
// POL: 0 = default-policy loads and stores; 1 = nontemporal loads, output through the sc1
// write-through buffer store; 2 = nontemporal loads and a nontemporal buffer store (the one
// workgroup-per-CU shape of long buckets, see launch_vec_chunk).
template <int N, int RULE, int U, int POL>
__global__ __launch_bounds__(kBlock) void mix_vec_kernel(float* out, Fanin f, long long nvec) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  // (unused and removed by the compiler when POL == 0)
  const __amdgpu_buffer_rsrc_t w =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<(POL != 0)>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 y = fold<N, RULE>(v[u], f);
      if constexpr (POL != 0)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y), w,
                                               (int)((base + (long long)u * kBlock) * 16), 0,
                                               POL == 2 ? kStoreNt : kStoreSc1);
      else
        st4<false>(out, base + (long long)u * kBlock, y);
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      f4 v[N + 1];
#pragma unroll
      for (int k = 0; k <= N; ++k) v[k] = ld4<false>(f.src[k], i);
      st4<false>(out, i, fold<N, RULE>(v, f));
    }
  }
}

// Vector mix + fused compression epilogue (count reduction per block). Tiles of kBlock * U
// float4 per block like mix_vec_kernel: U float4 of every stream per lane in flight together
// (U = 4 while (N + 1) * U <= 40 registers' worth of float4, as auto_vec), nontemporal loads.
// The epilogue's form (KIND, compress_sel) is a template parameter.
template <int N, int KIND>
__global__ __launch_bounds__(kBlock) void mix_vec_compress_kernel(float* out, Fanin f,
                                                                   long long nvec,
                                                                   CompressParams cp) {
  constexpr int U = (N + 1) * 4 <= 40 ? 4 : ((N + 1) * 2 <= 40 ? 2 : 1);
  constexpr long long kTile = (long long)kBlock * U;
  const Sc1Out o = sc1_out(out, nvec * 16);
  const float thr = (float)cp.thr, rep = (float)cp.rep;
  unsigned kept = 0;
  for (long long base = (long long)blockIdx.x * kTile + threadIdx.x; base < nvec;
       base += (long long)gridDim.x * kTile) {
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long i = base + (long long)u * kBlock;
        v[u][k] = i < nvec ? ld4<true>(f.src[k], i) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      if (i >= nvec) continue;
      f4 w = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      const long long e0 = i * 4;
      if (e0 + 3 >= cp.cbegin && e0 < cp.cend) {
        const f4 r = v[u][0];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const long long e = e0 + c;
          if (e >= cp.cbegin && e < cp.cend) w[c] = compress_sel<KIND>(w[c], r[c], thr, rep, kept);
        }
      }
      st16_sc1(o, i, w);
    }
  }
  block_add_count(kept, cp.kept);
}

// Scalar path: unaligned buckets and the <4-element tail.
struct ScalarFanin {
  const float* src[CFA_MAX_FANIN + 1];
  float c[CFA_MAX_FANIN + 1];
  float d[CFA_MAX_FANIN + 1];
  int n;
};
__global__ __launch_bounds__(kBlock) void mix_scalar_kernel(float* out, ScalarFanin f, long long P,
                                                            int rule, int compress,
                                                            CompressParams cp) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    const float w0 = f.src[0][i];
    float w;
    if (rule == CFA_RULE_SEQUENTIAL || rule == CFA_RULE_SEQUENTIAL_DIV) {
      w = w0;
      for (int j = 1; j <= f.n; ++j) {
        float t = f.src[j][i] - w;
        t = f.c[j] * t;
        if (rule == CFA_RULE_SEQUENTIAL_DIV) t = t / f.d[j];
        w = w + t;
      }
    } else {
      w = f.c[0] * w0;
      for (int j = 1; j <= f.n; ++j) w = fmaf(f.c[j], f.src[j][i], w);
    }
    if (compress && i >= cp.cbegin && i < cp.cend) w = compress_one(w, w0, cp, kept);
    out[i] = w;
  }
  if (compress) block_add_count(kept, cp.kept);
}

// Standalone compression epilogue (no mixing): y in place. Vectors [0, nvec) move 16 bytes per
// lane (y and ref 16-byte aligned), elements [4 * nvec, P) one at a time. The mode's form is a
// template parameter (compress_sel); full tiles of four float4 of y and ref per lane are walked
// grid-stride with no per-vector guards, the partial tile by one workgroup.
template <int KIND>
__global__ __launch_bounds__(kBlock) void compress_kernel(float* y, const float* ref, long long P,
                                                          long long nvec, CompressParams cp) {
  unsigned kept = 0;
  const float thr = (float)cp.thr, rep = (float)cp.rep;
  constexpr int U = 4;  // four float4 of y and ref per lane in flight together
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  f4* y4 = reinterpret_cast<f4*>(y);
  const f4* r4 = reinterpret_cast<const f4*>(ref);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // default-policy loads and stores: y is read and rewritten in place, and keeping its lines
      // in L2 between the two lets the store merge (13% faster than nontemporal, compress_sweep)
      v[u] = y4[base + (long long)u * kBlock];
      if constexpr (KIND == 2) r[u] = r4[base + (long long)u * kBlock];
      else r[u] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[u][c] = compress_sel<KIND>(v[u][c], r[u][c], thr, rep, kept);
      y4[base + (long long)u * kBlock] = v[u];  // in place: an sc1 store measured 20% slower, nt 13% slower
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      f4 v = y4[i];
      const f4 r = (KIND == 2) ? r4[i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = compress_sel<KIND>(v[c], r[c], thr, rep, kept);
      y4[i] = v;
    }
  }
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long i = 4 * nvec + (long long)blockIdx.x * kBlock + threadIdx.x; i < P; i += stride) {
    const float r = (KIND == 2) ? ref[i] : 0.0f;
    y[i] = compress_sel<KIND>(y[i], r, thr, rep, kept);
  }
  block_add_count(kept, cp.kept);
}

// ------------------------------------------------------------------------------------------
// Host-side dispatch.
// ------------------------------------------------------------------------------------------
template <int RULE, int U, int POL>
static void launch_vec_u(int n, unsigned grid, hipStream_t st, float* out, const Fanin& f,
                         long long nvec) {
#define CFA_CASE(K) \
  case K:           \
    mix_vec_kernel<K, RULE, U, POL><<<grid, kBlock, 0, st>>>(out, f, nvec); \
    break;
  switch (n) {
    CFA_CASE(0) CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6)
    CFA_CASE(7) CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13)
    CFA_CASE(14) CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
}

template <int RULE>
static void launch_vec_chunk(int n, hipStream_t st, float* out, const Fanin& f, long long nvec,
                             const cfa_launch_t& t);

template <int RULE>
static void launch_vec(int n, hipStream_t st, float* out, const Fanin& f, long long nvec,
                       const cfa_launch_t& t) {
  // chunks of at most kMaxChunkVec float4 (32-bit buffer offsets of the streaming store)
  for (long long done = 0; done < nvec; done += kMaxChunkVec) {
    const long long m = (nvec - done) < kMaxChunkVec ? (nvec - done) : kMaxChunkVec;
    Fanin g = f;
    for (int k = 0; k <= n; ++k) g.src[k] = f.src[k] + done * 4;
    launch_vec_chunk<RULE>(n, st, out + done * 4, g, m, t);
  }
}

template <int RULE>
static void launch_vec_chunk(int n, hipStream_t st, float* out, const Fanin& f, long long nvec,
                             const cfa_launch_t& t) {
  // library default (blocks_per_cu == kAutoBlocks): the mix's own shape, one workgroup per CU;
  // an explicit configuration (cfa_mix_seq_ex_f32, CFA_BLOCKS_PER_CU) keeps the round-1 auto vec
  // (the sequential rule only: the linear closed form measured 0.752 with it against 0.790 with
  // two workgroups x 4 float4 on the same buffers, profiles/r02_s3_kernel_rooflines_vec_same.jsonl)
  // The divisor fold (fp64-reciprocal division since round 4) takes the mix's shape too, with the
  // round-1 auto vec in the one-workgroup branch: at 25M, n = 8, one workgroup x four float4 ran
  // 0.776 of peak against 0.749 at two workgroups x one float4 (the Markstein form's shape) and
  // 0.760 at one x two (profiles/r04_div64_sweep.jsonl).
  const bool own = t.blocks_per_cu == kAutoBlocks &&
                   (RULE == CFA_RULE_SEQUENTIAL || RULE == CFA_RULE_SEQUENTIAL_DIV);
  int own_bpc = 1, own_vec = 1;
  if (own) mix_auto_shape(n, nvec, own_bpc, own_vec);
  if (own && RULE == CFA_RULE_SEQUENTIAL_DIV && own_bpc == 1) own_vec = auto_vec(n);
  const int U = t.vec_per_lane > 0 ? norm_vec(t.vec_per_lane) : (own ? own_vec : auto_vec(n));
  const long long tiles = (nvec + (long long)kBlock * U - 1) / ((long long)kBlock * U);
  cfa_launch_t shape = t;
  if (own) shape.blocks_per_cu = own_bpc;
  const unsigned grid = grid_for(tiles, shape);
  // Store policy (round 3, tools/probe/store_form.py and ab_store_r03.sh): with the one-workgroup
  // shape of buckets from 8M elements, a nontemporal store beats the sc1 write-through store
  // (25M, n = 8: 150.4 vs 152.1-153.1 us); at the four-workgroup shape of shorter buckets and
  // for the other rules' shapes the sc1 store stays ahead (3.125M: 17.8 vs 20.0 us).
  const bool nt_store = own && shape.blocks_per_cu == 1 && nvec * 4 >= (8LL << 20) && t.nontemporal;
  if (U == 4) {
    if (t.nontemporal) launch_vec_u<RULE, 4, 1>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 4, 0>(n, grid, st, out, f, nvec);
  } else if (U == 2) {
    if constexpr (RULE == CFA_RULE_SEQUENTIAL)
      if (nt_store) return launch_vec_u<RULE, 2, 2>(n, grid, st, out, f, nvec);
    if (t.nontemporal) launch_vec_u<RULE, 2, 1>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 2, 0>(n, grid, st, out, f, nvec);
  } else {
    if constexpr (RULE == CFA_RULE_SEQUENTIAL)
      if (nt_store) return launch_vec_u<RULE, 1, 2>(n, grid, st, out, f, nvec);
    if (t.nontemporal) launch_vec_u<RULE, 1, 1>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 1, 0>(n, grid, st, out, f, nvec);
  }
}

template <int KIND>
static void launch_vec_compress_k(int n, unsigned grid, hipStream_t st, float* out, const Fanin& f,
                                  long long nvec, const CompressParams& cp) {
#define CFA_CASE(K) \
  case K:           \
    mix_vec_compress_kernel<K, KIND><<<grid, kBlock, 0, st>>>(out, f, nvec, cp); \
    break;
  switch (n) {
    CFA_CASE(0) CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6)
    CFA_CASE(7) CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13)
    CFA_CASE(14) CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
}

static void launch_vec_compress(int n, hipStream_t st, float* out, const Fanin& f, long long nvec,
                                const CompressParams& cp) {
  const unsigned grid = grid_for((nvec + kBlock - 1) / kBlock);
  switch (compress_kind(cp.mode)) {
    case 1: launch_vec_compress_k<1>(n, grid, st, out, f, nvec, cp); break;
    case 2: launch_vec_compress_k<2>(n, grid, st, out, f, nvec, cp); break;
    default: launch_vec_compress_k<0>(n, grid, st, out, f, nvec, cp); break;
  }
}

// One pass of at most CFA_MAX_FANIN neighbours. Splits the bucket into a scalar head (until
// every pointer is 16-byte aligned, when they share the same misalignment), a float4 body and
// a scalar tail. Buckets with different misalignments run entirely on the scalar path.
static int mix_pass(float* out, const float* local, const float* const* nbrs, const float* c,
                    int n, size_t P, int rule, const CompressParams* cp, hipStream_t st,
                    const cfa_launch_t& lc = tune(), const float* div = nullptr) {
  const uintptr_t mis = addr(out) & 15;
  bool same = (addr(local) & 15) == mis;
  for (int j = 0; j < n; ++j) same = same && ((addr(nbrs[j]) & 15) == mis);
  const bool scalar_only = !same || (mis & 3) != 0;
  size_t head = 0, nvec = 0;
  if (!scalar_only) {
    head = mis ? (16 - mis) / 4 : 0;
    if (head > P) head = P;
    nvec = (P - head) / 4;
  } else {
    head = P;
  }
  const size_t tail_begin = head + nvec * 4;

  CompressParams cpv{};
  if (cp) cpv = *cp;

  if (nvec > 0) {
    Fanin f{};
    f.src[0] = local + head;
    for (int j = 0; j < n; ++j) f.src[j + 1] = nbrs[j] + head;
    for (int k = 0; k <= n; ++k) f.c[k] = c[k];
    for (int k = 0; k <= n; ++k) f.d[k] = div ? div[k] : 1.0f;
    set_reciprocals(f, n);
    if (cp) {
      CompressParams shifted = cpv;
      shifted.cbegin = cpv.cbegin - (long long)head;
      shifted.cend = cpv.cend - (long long)head;
      launch_vec_compress(n, st, out + head, f, (long long)nvec, shifted);
    } else if (rule == CFA_RULE_SEQUENTIAL) {
      launch_vec<CFA_RULE_SEQUENTIAL>(n, st, out + head, f, (long long)nvec, lc);
    } else if (rule == CFA_RULE_SEQUENTIAL_DIV) {
      launch_vec<CFA_RULE_SEQUENTIAL_DIV>(n, st, out + head, f, (long long)nvec, lc);
    } else {
      launch_vec<CFA_RULE_LINEAR>(n, st, out + head, f, (long long)nvec, lc);
    }
    if (int rc = check_launch("mix_vec")) return rc;
  }
  // Scalar pieces: [0, head) and [tail_begin, P).
  const size_t pieces[2][2] = {{0, head}, {tail_begin, P}};
  for (auto& pc : pieces) {
    const size_t b = pc[0], e = pc[1];
    if (e <= b) continue;
    ScalarFanin sf{};
    sf.src[0] = local + b;
    for (int j = 0; j < n; ++j) {
      sf.src[j + 1] = nbrs[j] + b;
    }
    for (int k = 0; k <= n; ++k) sf.c[k] = c[k];
    for (int k = 0; k <= n; ++k) sf.d[k] = div ? div[k] : 1.0f;
    sf.n = n;
    CompressParams sc = cpv;
    sc.cbegin = cpv.cbegin - (long long)b;
    sc.cend = cpv.cend - (long long)b;
    const long long len = (long long)(e - b);
    mix_scalar_kernel<<<grid_for((len + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        out + b, sf, len, rule, cp ? 1 : 0, sc);
    if (int rc = check_launch("mix_scalar")) return rc;
  }
  return CFA_OK;
}

// Sequential rule over any fan-in: chunks of CFA_MAX_FANIN; chunk k>0 continues from `out`.
// The compression epilogue is fused into the (single) pass when n <= CFA_MAX_FANIN; wider
// fan-ins run it as a separate pass with the untouched pre-mix `local` as DPCM reference.
static int mix_seq_any(float* out, const float* local, const float* const* nbrs,
                       const float* alphas, int n, size_t P, const CompressParams* cp,
                       hipStream_t st, const cfa_launch_t& lc = tune()) {
  if (int rc = validate_mix(out, local, nbrs, n, P)) return rc;
  if (P == 0) return CFA_OK;
  const bool split_epilogue = cp && n > CFA_MAX_FANIN;
  if (split_epilogue && out == local && needs_ref(cp->mode))
    return fail(CFA_E_INVALID, "in-place DPCM compression needs fan-in <= %d", CFA_MAX_FANIN);
  int done = 0;
  const float* w = local;
  float c[CFA_MAX_FANIN + 1];
  do {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    c[0] = 1.0f;
    for (int j = 0; j < m; ++j) c[j + 1] = alphas[done + j];
    const CompressParams* fused = (cp && !split_epilogue) ? cp : nullptr;
    if (int rc = mix_pass(out, w, nbrs + done, c, m, P, CFA_RULE_SEQUENTIAL, fused, st, lc))
      return rc;
    done += m;
    w = out;
  } while (done < n);
  if (split_epilogue)
    return cfa_compress_epilogue_f32(out + cp->cbegin, local + cp->cbegin, cp->mode,
                                     (size_t)(cp->cend - cp->cbegin), cp->kept, st);
  return CFA_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
extern "C" int cfa_mix_seq_f32(float* out, const float* local, const float* const* nbrs,
                               const float* alphas, int n, size_t P, void* stream) {
  if (n > 0 && !alphas) return fail(CFA_E_INVALID, "null alphas");
  return mix_seq_any(out, local, nbrs, alphas, n, P, nullptr, (hipStream_t)stream);
}

extern "C" int cfa_mix_seq_ex_f32(float* out, const float* local, const float* const* nbrs,
                                  const float* alphas, int n, size_t P,
                                  const cfa_launch_t* launch, void* stream) {
  if (n > 0 && !alphas) return fail(CFA_E_INVALID, "null alphas");
  if (launch && launch->blocks_per_cu < 0) return fail(CFA_E_INVALID, "blocks_per_cu < 0");
  cfa_launch_t lc = launch ? *launch : tune();
  lc.vec_per_lane = norm_vec(lc.vec_per_lane);
  return mix_seq_any(out, local, nbrs, alphas, n, P, nullptr, (hipStream_t)stream, lc);
}

extern "C" int cfa_mix_seq_div_f32(float* out, const float* local, const float* const* nbrs,
                                   const float* alphas, const float* divisors, int n, size_t P,
                                   void* stream) {
  if (n > 0 && (!alphas || !divisors)) return fail(CFA_E_INVALID, "null alphas/divisors");
  if (int rc = validate_mix(out, local, nbrs, n, P)) return rc;
  if (P == 0) return CFA_OK;
  hipStream_t st = (hipStream_t)stream;
  int done = 0;
  const float* w = local;
  float c[CFA_MAX_FANIN + 1], d[CFA_MAX_FANIN + 1];
  do {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    c[0] = 1.0f;
    d[0] = 1.0f;
    for (int j = 0; j < m; ++j) {
      c[j + 1] = alphas[done + j];
      d[j + 1] = divisors[done + j];
    }
    if (int rc = mix_pass(out, w, nbrs + done, c, m, P, CFA_RULE_SEQUENTIAL_DIV, nullptr, st,
                          tune(), d))
      return rc;
    done += m;
    w = out;
  } while (done < n);
  return CFA_OK;
}

extern "C" int cfa_mix_f32(float* out, const float* local, const float* const* nbrs,
                           const float* coeff, int n, size_t P, void* stream) {
  if (!coeff) return fail(CFA_E_INVALID, "null coefficients");
  if (int rc = validate_mix(out, local, nbrs, n, P)) return rc;
  if (P == 0) return CFA_OK;
  hipStream_t st = (hipStream_t)stream;
  int done = 0;
  const float* w = local;
  float c[CFA_MAX_FANIN + 1];
  do {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    c[0] = done == 0 ? coeff[0] : 1.0f;
    for (int j = 0; j < m; ++j) c[j + 1] = coeff[done + j + 1];
    if (int rc = mix_pass(out, w, nbrs + done, c, m, P, CFA_RULE_LINEAR, nullptr, st)) return rc;
    done += m;
    w = out;
  } while (done < n);
  return CFA_OK;
}

extern "C" int cfa_mix_seq_compress_f32(float* out, const float* local, const float* const* nbrs,
                                        const float* alphas, int n, size_t P, int mode,
                                        size_t cbegin, size_t cend,
                                        unsigned long long* kept_count, void* stream) {
  if (n > 0 && !alphas) return fail(CFA_E_INVALID, "null alphas");
  if (!kept_count) return fail(CFA_E_INVALID, "null kept_count");
  if (cbegin > cend || cend > P) return fail(CFA_E_INVALID, "bad compression range");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  cp.cbegin = (long long)cbegin;
  cp.cend = (long long)cend;
  cp.kept = kept_count;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    // No neighbours: out = local, then the epilogue (TF1/consensus/cfa_ongraphs.py:218-223).
    if (out != local && P > 0)
      CFA_HIP_CHECK(hipMemcpyAsync(out, local, P * sizeof(float), hipMemcpyDefault, st));
    return cfa_compress_epilogue_f32(out + cbegin, local + cbegin, mode, cend - cbegin,
                                     kept_count, stream);
  }
  return mix_seq_any(out, local, nbrs, alphas, n, P, &cp, st);
}

extern "C" int cfa_compress_epilogue_f32(float* y, const float* ref, int mode, size_t P,
                                         unsigned long long* kept_count, void* stream) {
  if (!kept_count) return fail(CFA_E_INVALID, "null kept_count");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  if ((mode == CFA_COMPRESS_SPARSE_DPCM || mode == CFA_COMPRESS_SPARSE_DPCM_HI) && !ref && P)
    return fail(CFA_E_INVALID, "DPCM compression needs a reference bucket");
  if (P == 0) return CFA_OK;
  if (!y) return fail(CFA_E_INVALID, "null bucket");
  cp.cbegin = 0;
  cp.cend = (long long)P;
  cp.kept = kept_count;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (addr(y) & 15) == 0 && (!ref || (addr(ref) & 15) == 0);
  const long long nvec = vec ? (long long)P / 4 : 0;
  const unsigned grid = grid_for(((vec ? nvec : (long long)P) + kBlock - 1) / kBlock);
  switch (compress_kind(mode)) {
    case 1: compress_kernel<1><<<grid, kBlock, 0, st>>>(y, ref, (long long)P, nvec, cp); break;
    case 2: compress_kernel<2><<<grid, kBlock, 0, st>>>(y, ref, (long long)P, nvec, cp); break;
    default: compress_kernel<0><<<grid, kBlock, 0, st>>>(y, ref, (long long)P, nvec, cp); break;
  }
  return check_launch("compress");
}

