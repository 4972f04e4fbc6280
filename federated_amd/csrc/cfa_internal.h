// cfa_internal.h — shared internals of libcfa's translation units (not installed, not an ABI).
//
// Device helpers for gfx950 (MI355X / CDNA4): the float4 streaming loads and stores, the fold of
// the sequential / linear / FedAvg rules, the compression epilogue, the launch-shape defaults,
// and the thread-local error reporting behind cfa_last_error(). Every .hip file of the library
// is compiled with -ffp-contract=off: CFA_RULE_SEQUENTIAL evaluates t = x - w; t = a * t;
// w = w + t exactly as fp32 numpy does (three roundings), which makes the TF2 path
// bit-identical to the reference; CFA_RULE_LINEAR uses explicit fmaf.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "cfa_engine.h"

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// Error reporting: one thread-local message per thread, shared by the library's translation
// units (C++17 inline variable); no global mutable state is shared between threads.
// ------------------------------------------------------------------------------------------
inline thread_local std::string g_last_error;

__attribute__((format(printf, 2, 3))) inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define CFA_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(CFA_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                  __FILE__, __LINE__);                                                   \
  } while (0)

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CFA_E_HIP, "%s launch failed: %s", what, hipGetErrorString(e));
  return CFA_OK;
}

namespace {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Default launch configuration (cfa_launch_t), optionally overridden once from the
// environment (CFA_BLOCKS_PER_CU, CFA_VEC_PER_LANE, CFA_NONTEMPORAL); immutable after first use.
// Explicit per-call configurations go through cfa_mix_seq_ex_f32.
// Defaults from the in-process sweep on MI355X (tools/tune_mix.py, profiles/r01_tune.jsonl):
// 2 resident workgroups per CU with a grid-stride loop, nontemporal loads and stores, and
// vec_per_lane = 0 (auto: the widest tile that keeps (n+1)*vec <= 40 float4 in registers); the
// streaming mix kernel has its own default below.
// blocks_per_cu = kAutoBlocks in the library default means "per kernel": the streaming mix
// kernel takes its own shape (mix_auto_shape), every other kernel kDefaultBlocks.
constexpr int kDefaultBlocks = 2;
constexpr int kAutoBlocks = -1;
static int norm_vec(int v) { return v >= 4 ? 4 : (v >= 2 ? 2 : (v == 1 ? 1 : 0)); }
static int auto_vec(int n) { return (n + 1) * 4 <= 40 ? 4 : ((n + 1) * 2 <= 40 ? 2 : 1); }
// The streaming mix's own default (round 2, tools/probe/tune_placed.py on placement-calibrated
// stacks, profiles/r02_tune_placed.jsonl: every shape of 1-4 workgroups per CU x 1/2/4 float4 per
// lane at K = 2/4/8/12 on two boxes): one workgroup per CU (one wave per SIMD) at every fan-in,
// two float4 per lane except for 3-5 neighbours, where one is best. Sequential rule only.
static int mix_auto_vec(int n) { return (n >= 3 && n <= 5) ? 1 : ((n + 1) * 2 <= 40 ? 2 : 1); }
// ... for buckets of 8M elements and more. Shorter mixes need more loads in flight than one
// wave per SIMD issues (round 3, tools/probe/slice_shape.py on placement-calibrated populations,
// P = 0.5M-25M; profiles/r03_slice_shape_k{4,8}.jsonl for the sweep, r03_ab_shape.jsonl for two
// rounds of A/B against the one-workgroup shape at K = 2/4/8/16). Four workgroups per CU:
//   - with one float4 per lane from 512K to 1.5M elements (1M: +2-13% in 3 of 4 A/B pairs);
//   - with four float4 from 1.5M to 8M (3.125M, the N = 8 bench rank's slice: +6-13% on ring
//     windows, +7% on rows no two consecutive mixes share; 6.25M: +1-5%);
//   - with two for 10-16 neighbours from 1.5M to 3M (+3-5%; neutral to -2% above).
// Below 512K elements (e.g. the drop-in pipeline's 128K chunks read over PCIe; at 500K the A/B
// pairs split both ways at K = 4 and 16) the shape is unchanged.
static void mix_auto_shape(int n, long long nvec, int& blocks_per_cu, int& vec) {
  const long long elems = nvec * 4;
  const bool narrow = (n + 1) * 4 <= 40;
  blocks_per_cu = 4;
  if (elems >= (1LL << 19) && elems < (3LL << 19)) {
    vec = 1;
  } else if (elems >= (3LL << 19) && elems < (8LL << 20) && narrow) {
    vec = 4;
  } else if (elems >= (3LL << 19) && elems < (3LL << 20) && !narrow) {
    vec = 2;
  } else {
    blocks_per_cu = 1;
    vec = mix_auto_vec(n);
  }
}
static cfa_launch_t read_tune() {
  cfa_launch_t t{kAutoBlocks, 0, 1};
  if (const char* s = getenv("CFA_BLOCKS_PER_CU")) {
    const int v = atoi(s);  // 0 = one workgroup per tile, > 0 = cap per CU; negative = the default
    t.blocks_per_cu = v >= 0 ? v : kAutoBlocks;
  }
  if (const char* s = getenv("CFA_VEC_PER_LANE")) t.vec_per_lane = norm_vec(atoi(s));
  if (const char* s = getenv("CFA_NONTEMPORAL")) t.nontemporal = atoi(s) ? 1 : 0;
  return t;
}
static const cfa_launch_t& tune() {
  static const cfa_launch_t t = read_tune();  // C++11 magic static: thread-safe init
  // CFA_TUNE_DYNAMIC=1 (measurement tools only): re-read the environment at every launch, so one
  // process can compare launch shapes on the same buffers (tools/probe/tune_entries.py)
  static const bool dynamic = getenv("CFA_TUNE_DYNAMIC") != nullptr;
  if (dynamic) {
    thread_local cfa_launch_t d;
    d = read_tune();
    return d;
  }
  return t;
}

}  // namespace

// Per-device CU count, cached after the first query. An inline function with external linkage,
// so every translation unit shares one cache; cfa_device_prepare() fills it before any launch
// (the launch path then only reads it, which keeps hipGraph capture free of device queries).
inline int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < 64) {
    const int c = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (c > 0) return c;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return 256;
  if (dev >= 0 && dev < 64) __atomic_store_n(&cache[dev], cus, __ATOMIC_RELAXED);
  return cus;
}

// cfa_grad.hip: per-device LDS query and kernel LDS limits, done ahead of any capture.
int grad_prepare_device();

namespace {

static unsigned grid_for(long long tiles, const cfa_launch_t& t = tune()) {
  if (tiles <= 0) return 1;
  long long g = tiles;
  const int bpc = t.blocks_per_cu == kAutoBlocks ? kDefaultBlocks : t.blocks_per_cu;
  if (bpc > 0) {
    long long cap = (long long)device_cus() * bpc;
    if (g > cap) g = cap;
  }
  if (g > 0x7fffffffLL) g = 0x7fffffffLL;
  return (unsigned)g;
}

// grid_for with a kernel's own default workgroups per CU, used while the launch configuration is
// the library default (an explicit CFA_BLOCKS_PER_CU applies to every kernel alike).
static unsigned grid_for_own(long long tiles, int own_blocks_per_cu) {
  cfa_launch_t t = tune();
  if (t.blocks_per_cu == kAutoBlocks) t.blocks_per_cu = own_blocks_per_cu;
  return grid_for(tiles, t);
}

// Kernel-argument pack: pointers + coefficients land in SGPRs.
struct Fanin {
  const float* src[CFA_MAX_FANIN + 1];  // [0] = local (w0), [1..N] = neighbours
  float c[CFA_MAX_FANIN + 1];           // SEQ: c[j] = alpha of src[j] (c[0] unused); LIN: coeff
  float d[CFA_MAX_FANIN + 1];           // SEQ_DIV: d[j] = divisor of step j (d[0] unused)
  double rd[CFA_MAX_FANIN + 1];         // SEQ_DIV: rd[j] = RN_64(1 / d[j]) (div4_rn)
};

// Correctly rounded fp32 a / b as one fp64 multiply: q = (float)((double)a * RN_64(1/b)) is IEEE
// a / b whenever the exact quotient is not an exact SUBNORMAL rounding midpoint. Away from a
// midpoint the exact quotient of two 24-bit significands lies at least 2^-48 (relative) from it,
// while the two fp64 roundings (of 1/b and of the product) stay within 2^-52: the conversion
// rounds the right way, normal or subnormal, and fp64's exponent range holds every fp32 quotient
// (overflow happens in the conversion as in the IEEE division; zeros, infinities and NaN
// propagate as there). A subnormal quotient has fewer significand bits and CAN sit exactly on a
// midpoint (a = odd k * o * 2^-149, b = 2o): there the fp64 error of RN(1/b) decides the rounding
// instead of ties-to-even (round-4 advisor finding). Such a quotient converts to a subnormal fp32
// (or to 0 only when it is below the 2^-150 tie, which rounds to 0 anyway; the tie below 2^-126
// rounds up to the normal 2^-126, which ties-to-even also gives), so each step records whether
// any of its results is subnormal (one v_cmp_class per element, OR-ed on the scalar unit), and a
// fold that saw one redoes its tile with the IEEE division (fold below: one exec-masked branch per
// tile, never taken on the bench's buckets). Round 4 replaced Markstein's three fp32 operations
// plus a range test per float4 with the one-multiply form (profiles/r04_div64_sweep.jsonl: 0.733
// -> 0.776 of peak at 25M, n = 8). Tested bit for bit against numpy over every binade and on exact
// subnormal ties (tests/test_gpu_kernels.py test_mix_seq_div_*; the rule itself on the CPU,
// tests/test_div64_rule.py).
constexpr int kFcSubnormal = 0x0090;  // __builtin_isfpclass: negative | positive subnormal
__device__ __forceinline__ f4 div4_rn(f4 a, double rb, bool& subnormal) {
  f4 q;
  q.x = (float)((double)a.x * rb);
  q.y = (float)((double)a.y * rb);
  q.z = (float)((double)a.z * rb);
  q.w = (float)((double)a.w * rb);
  subnormal = subnormal | __builtin_isfpclass(q.x, kFcSubnormal) | __builtin_isfpclass(q.y, kFcSubnormal) |
              __builtin_isfpclass(q.z, kFcSubnormal) | __builtin_isfpclass(q.w, kFcSubnormal);
  return q;
}
__device__ __forceinline__ f4 div4_ieee(f4 a, float b) {
  f4 q;
  q.x = a.x / b;
  q.y = a.y / b;
  q.z = a.z / b;
  q.w = a.w / b;
  return q;
}

// Host side: fills f.rd from f.d[0..n].
inline void set_reciprocals(Fanin& f, int n) {
  for (int k = 0; k <= n; ++k) f.rd[k] = 1.0 / (double)f.d[k];
}

template <bool NT>
__device__ __forceinline__ f4 ld4(const float* p, long long i) {
  const f4* q = reinterpret_cast<const f4*>(p) + i;
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, long long i, f4 v) {
  f4* q = reinterpret_cast<f4*>(p) + i;
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

template <int N, int RULE>
__device__ __forceinline__ f4 fold(const f4 (&v)[N + 1], const Fanin& f) {
  if constexpr (RULE == CFA_RULE_SEQUENTIAL) {
    f4 w = v[0];
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      f4 t = v[j] - w;  // numpy: (x - w)
      t = f.c[j] * t;   //        eps * (...)
      w = w + t;        //        w + (...)
    }
    return w;
  } else if constexpr (RULE == CFA_RULE_SEQUENTIAL_DIV) {
    f4 w = v[0];
    bool subnormal = false;
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      f4 t = v[j] - w;  // numpy: (x - w)
      t = f.c[j] * t;   //        u * (...)
      t = div4_rn(t, f.rd[j], subnormal);  // (...) / C, one fp64 multiply
      w = w + t;
    }
    if (__builtin_expect(subnormal, 0)) {  // a subnormal quotient may be an exact tie: IEEE division
      w = v[0];
#pragma unroll
      for (int j = 1; j <= N; ++j) {
        f4 t = v[j] - w;
        t = f.c[j] * t;
        t = div4_ieee(t, f.d[j]);
        w = w + t;
      }
    }
    return w;
  } else {
    f4 w = f.c[0] * v[0];
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      w.x = fmaf(f.c[j], v[j].x, w.x);
      w.y = fmaf(f.c[j], v[j].y, w.y);
      w.z = fmaf(f.c[j], v[j].z, w.z);
      w.w = fmaf(f.c[j], v[j].w, w.w);
    }
    return w;
  }
}

// Compression epilogue on one element (TF1/consensus/cfa_ongraphs.py:225-273), fp32 arrays.
// numpy 2 (NEP 50) casts the Python-float threshold and replacement to fp32, so the test, the
// product sign(.)*rep and the DPCM sum ref + sign(.)*rep are all fp32 operations (the reference
// reaches this with fp32 arrays when a call has no neighbour, :218-223). sign(0) = 0 and
// sign(NaN) = NaN as numpy. The fp64 variant (compress_one_d) serves the fp64 chains.
__device__ __forceinline__ double np_sign(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x);
}
__device__ __forceinline__ float np_signf(float x) {
  return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : x);
}
struct CompressParams {
  int mode;
  double thr, rep;
  long long cbegin, cend;  // element range the epilogue applies to
  unsigned long long* kept;
};
__device__ __forceinline__ float compress_one(float y, float ref, const CompressParams& cp,
                                              unsigned& kept) {
  const float thr = (float)cp.thr, rep = (float)cp.rep;
  if (cp.mode == CFA_COMPRESS_SPARSE || cp.mode == CFA_COMPRESS_SPARSE_HI) {
    if (fabsf(y) < thr) return np_signf(y) * rep;
  } else if (cp.mode == CFA_COMPRESS_SPARSE_DPCM || cp.mode == CFA_COMPRESS_SPARSE_DPCM_HI) {
    const float d = y - ref;
    if (fabsf(d) < thr) return ref + np_signf(d) * rep;
  }
  ++kept;
  return y;
}

// The same epilogue with the mode's form fixed at compile time (KIND: 0 none, 1 sparse, 2 DPCM;
// compress_kind maps a mode to it) and the thresholds passed in as fp32: straight-line selects
// instead of a per-element branch tree on the runtime mode, which kept the standalone epilogue's
// waves off the memory pipe between tiles (round 4, tools/probe/lowrow_sweep.py). The same fp32
// operations as compress_one, so the same values and count.
__device__ __host__ constexpr int compress_kind(int mode) {
  return (mode == CFA_COMPRESS_SPARSE || mode == CFA_COMPRESS_SPARSE_HI) ? 1
         : (mode == CFA_COMPRESS_SPARSE_DPCM || mode == CFA_COMPRESS_SPARSE_DPCM_HI) ? 2 : 0;
}
template <int KIND>
__device__ __forceinline__ float compress_sel(float y, float ref, float thr, float rep, unsigned& kept) {
  if constexpr (KIND == 0) {
    ++kept;
    return y;
  } else {
    const float d = KIND == 2 ? y - ref : y;
    const bool hit = fabsf(d) < thr;
    const float r = KIND == 2 ? ref + np_signf(d) * rep : np_signf(y) * rep;
    kept += hit ? 0u : 1u;
    return hit ? r : y;
  }
}

// Block-wide sum of one counter per lane, then a single 64-bit atomic per block.
__device__ __forceinline__ void block_add_count(unsigned kept, unsigned long long* dst) {
  __shared__ unsigned red[kBlock / 64];
  unsigned v = kept;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; ++i) s += red[i];
    if (s) atomicAdd(dst, s);
  }
}


// Streaming-policy store (NT kernels): write-through with sc1, so the once-written output does
// not leave dirty lines in the XCD's L2 (measured +3% over an nt store on the mix kernel at two
// workgroups per CU, tools/tune_cache_policy.py); the sequential mix's one-workgroup shape of long
// buckets stores nontemporally instead (kStoreNt, +1%, tools/probe/ab_store_r03.sh). Buffer
// stores take 32-bit offsets: the host splits a vector body into launches of at most kMaxChunkVec
// float4 (2 GiB).
constexpr long long kMaxChunkVec = 1LL << 27;
constexpr int kStoreSc1 = 16;
constexpr int kStoreNt = 2;

// Streaming store of one 16-byte vector with the sc1 write-through policy, as the headline mix
// stores its output (kStoreSc1): through a buffer resource when every byte offset of the output
// fits the 31 bits the kernels pass, else a nontemporal global store. The choice is uniform per
// launch (one scalar branch).
struct Sc1Out {
  __amdgpu_buffer_rsrc_t r;
  void* base;
  bool buf;
};
__device__ __forceinline__ Sc1Out sc1_out(void* base, long long bytes) {
  Sc1Out o;
  o.base = base;
  o.buf = bytes <= 0x7FFFFFF0LL;
  o.r = __builtin_amdgcn_make_buffer_rsrc(base, 0, o.buf ? (unsigned)bytes : 0u, 0x00020000);
  return o;
}
template <typename V>
__device__ __forceinline__ void st16_sc1(const Sc1Out& o, long long idx, V v) {  // idx: 16-byte units
  static_assert(sizeof(V) == 16, "16-byte vectors only");
  if (o.buf)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), o.r, (int)(idx * 16), 0, kStoreSc1);
  else
    __builtin_nontemporal_store(v, reinterpret_cast<V*>(o.base) + idx);
}

// fp64 form of the epilogue for the fp64 chains (TF1 W_up_l2 is fp64 in the reference).
__device__ __forceinline__ double compress_one_d(double y, double ref, const CompressParams& cp,
                                                 unsigned& kept) {
  if (cp.mode == CFA_COMPRESS_SPARSE || cp.mode == CFA_COMPRESS_SPARSE_HI) {
    if (fabs(y) < cp.thr) return np_sign(y) * cp.rep;
  } else if (cp.mode == CFA_COMPRESS_SPARSE_DPCM || cp.mode == CFA_COMPRESS_SPARSE_DPCM_HI) {
    const double d = y - ref;
    if (fabs(d) < cp.thr) return ref + np_sign(d) * cp.rep;
  }
  ++kept;
  return y;
}

static inline uintptr_t addr(const void* p) { return reinterpret_cast<uintptr_t>(p); }

static int compress_params(int mode, CompressParams& cp) {
  cp.mode = mode;
  switch (mode) {
    case CFA_COMPRESS_NONE: cp.thr = 0.0; cp.rep = 0.0; break;
    case CFA_COMPRESS_SPARSE: cp.thr = 0.001; cp.rep = 0.0001; break;
    case CFA_COMPRESS_SPARSE_DPCM: cp.thr = 1.e-4; cp.rep = 1.e-4; break;
    case CFA_COMPRESS_SPARSE_DPCM_HI: cp.thr = 1.e-3; cp.rep = 1.e-3; break;
    case CFA_COMPRESS_SPARSE_HI: cp.thr = 0.01; cp.rep = 0.001; break;
    default: return fail(CFA_E_INVALID, "unknown compression mode %d", mode);
  }
  return CFA_OK;
}

static int validate_mix(const float* out, const float* local, const float* const* nbrs, int n,
                        size_t P) {
  if (n < 0) return fail(CFA_E_INVALID, "negative fan-in %d", n);
  if (P == 0) return CFA_OK;
  if (!out || !local) return fail(CFA_E_INVALID, "null out/local bucket");
  if (n > 0 && !nbrs) return fail(CFA_E_INVALID, "null neighbour table");
  for (int j = 0; j < n; ++j) {
    if (!nbrs[j]) return fail(CFA_E_INVALID, "null neighbour bucket %d", j);
    if (nbrs[j] == out) return fail(CFA_E_INVALID, "output aliases neighbour %d", j);
  }
  return CFA_OK;
}

static bool needs_ref(int mode) {
  return mode == CFA_COMPRESS_SPARSE_DPCM || mode == CFA_COMPRESS_SPARSE_DPCM_HI;
}
}  // namespace
