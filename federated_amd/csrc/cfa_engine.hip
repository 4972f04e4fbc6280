// cfa_engine.hip — gfx950 (MI355X / CDNA4) kernels + C-ABI for CFA / CFA-GE consensus mixing.
//
// The reference computes the mixing step as numpy AXPY chains over whole tensors, one
// neighbour at a time, with a file round trip between neighbours:
//   TF1/consensus/cfa.py:66-76, cfa_ongraphs.py:109-119, cfa_ge_2stage.py:73-83 / 594-621,
//   TF2 consensus_v3.py:153-155, consensus_v4.py:211-213 / 251-253.
// Here one launch folds every neighbour of a device in registers: each lane streams one
// 16-byte slice of the local bucket and of all n neighbour buckets from HBM, applies the
// rule, and writes the result once. The work is HBM-bound (0.2-0.45 flop/byte), so there is
// no MFMA and no LDS data staging: the mixing coefficients and the bucket pointers live in
// the kernel arguments (SGPRs), loads are 16 B/lane (global_load_dwordx4), every load of a
// tile is issued before the first use, and the fan-in N is a template parameter so the
// fold is fully unrolled.
//
// Numerics: this file is compiled with -ffp-contract=off. CFA_RULE_SEQUENTIAL evaluates
// t = x - w; t = a * t; w = w + t exactly as fp32 numpy does (three roundings), which makes
// the TF2 path bit-identical to the reference. CFA_RULE_LINEAR uses explicit fmaf.
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

// ------------------------------------------------------------------------------------------
// Error reporting (thread-local, no global mutable state shared between threads).
// ------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
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

static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CFA_E_HIP, "%s launch failed: %s", what, hipGetErrorString(e));
  return CFA_OK;
}

extern "C" int cfa_version(void) { return CFA_VERSION; }
extern "C" const char* cfa_last_error(void) { return g_last_error.c_str(); }
// Used by cfa_comm.cpp so both translation units report through one thread-local message.
extern "C" __attribute__((visibility("hidden"))) void cfa_internal_set_error(const char* msg) {
  g_last_error = msg ? msg : "";
}

namespace {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

// Default launch configuration (cfa_launch_t), optionally overridden once from the
// environment (CFA_BLOCKS_PER_CU, CFA_VEC_PER_LANE, CFA_NONTEMPORAL); immutable after first use.
// Explicit per-call configurations go through cfa_mix_seq_ex_f32.
// Defaults from the in-process sweep on MI355X (tools/tune_mix.py, profiles/r01_tune.jsonl):
// 2 resident workgroups per CU with a grid-stride loop, nontemporal loads and stores, and
// vec_per_lane = 0 (auto: the widest tile that keeps (n+1)*vec <= 40 float4 in registers).
static int norm_vec(int v) { return v >= 4 ? 4 : (v >= 2 ? 2 : (v == 1 ? 1 : 0)); }
static int auto_vec(int n) { return (n + 1) * 4 <= 40 ? 4 : ((n + 1) * 2 <= 40 ? 2 : 1); }
static cfa_launch_t read_tune() {
  cfa_launch_t t{2, 0, 1};
  if (const char* s = getenv("CFA_BLOCKS_PER_CU")) t.blocks_per_cu = atoi(s);
  if (const char* s = getenv("CFA_VEC_PER_LANE")) t.vec_per_lane = norm_vec(atoi(s));
  if (const char* s = getenv("CFA_NONTEMPORAL")) t.nontemporal = atoi(s) ? 1 : 0;
  return t;
}
static const cfa_launch_t& tune() {
  static const cfa_launch_t t = read_tune();  // C++11 magic static: thread-safe init
  return t;
}

static int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return 256;
  return cus;
}

static unsigned grid_for(long long tiles, const cfa_launch_t& t = tune()) {
  if (tiles <= 0) return 1;
  long long g = tiles;
  if (t.blocks_per_cu > 0) {
    long long cap = (long long)device_cus() * t.blocks_per_cu;
    if (g > cap) g = cap;
  }
  if (g > 0x7fffffffLL) g = 0x7fffffffLL;
  return (unsigned)g;
}

// Kernel-argument pack: pointers + coefficients land in SGPRs.
struct Fanin {
  const float* src[CFA_MAX_FANIN + 1];  // [0] = local (w0), [1..N] = neighbours
  float c[CFA_MAX_FANIN + 1];           // SEQ: c[j] = alpha of src[j] (c[0] unused); LIN: coeff
  float d[CFA_MAX_FANIN + 1];           // SEQ_DIV: d[j] = divisor of step j (d[0] unused)
};

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
#pragma unroll
    for (int j = 1; j <= N; ++j) {
      f4 t = v[j] - w;  // numpy: (x - w)
      t = f.c[j] * t;   //        u * (...)
      t = t / f.d[j];   //        (...) / C   (IEEE-correct fp32 division)
      w = w + t;
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

// ------------------------------------------------------------------------------------------
// Vector mix kernel: tiles of kBlock*U float4 per block, grid-stride over tiles; the last
// partial tile is handled with per-vector guards by the block that owns it.
// ------------------------------------------------------------------------------------------
// Streaming-policy store (NT kernels): write-through with sc1, so the once-written output does
// not leave dirty lines in the XCD's L2 (measured +3% over an nt store on this kernel,
// tools/tune_cache_policy.py). Buffer stores take 32-bit offsets: the host splits the vector
// body into launches of at most kMaxChunkVec float4 (2 GiB).
typedef unsigned u4v __attribute__((ext_vector_type(4)));
constexpr long long kMaxChunkVec = 1LL << 27;
constexpr int kStoreSc1 = 16;

template <int N, int RULE, int U, bool NT>
__global__ __launch_bounds__(kBlock) void mix_vec_kernel(float* out, Fanin f, long long nvec) {
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  // (unused and removed by the compiler when !NT)
  const __amdgpu_buffer_rsrc_t w =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u][k] = ld4<NT>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 y = fold<N, RULE>(v[u], f);
      if constexpr (NT)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y), w,
                                               (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
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

// Vector mix + fused compression epilogue (count reduction per block).
template <int N>
__global__ __launch_bounds__(kBlock) void mix_vec_compress_kernel(float* out, Fanin f,
                                                                   long long nvec,
                                                                   CompressParams cp) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec;
       i += (long long)gridDim.x * kBlock) {
    f4 v[N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k) v[k] = ld4<false>(f.src[k], i);
    f4 w = fold<N, CFA_RULE_SEQUENTIAL>(v, f);
    const long long e0 = i * 4;
    if (e0 + 3 >= cp.cbegin && e0 < cp.cend) {
      const f4 r = v[0];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const long long e = e0 + c;
        if (e >= cp.cbegin && e < cp.cend) w[c] = compress_one(w[c], r[c], cp, kept);
      }
    }
    st4<false>(out, i, w);
  }
  block_add_count(kept, cp.kept);
}

// Scalar path: unaligned buckets, the <4-element tail, and strided neighbours.
struct ScalarFanin {
  const float* src[CFA_MAX_FANIN + 1];
  long long stride[CFA_MAX_FANIN + 1];
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
    const float w0 = f.src[0][i * f.stride[0]];
    float w;
    if (rule == CFA_RULE_SEQUENTIAL || rule == CFA_RULE_SEQUENTIAL_DIV) {
      w = w0;
      for (int j = 1; j <= f.n; ++j) {
        float t = f.src[j][i * f.stride[j]] - w;
        t = f.c[j] * t;
        if (rule == CFA_RULE_SEQUENTIAL_DIV) t = t / f.d[j];
        w = w + t;
      }
    } else {
      w = f.c[0] * w0;
      for (int j = 1; j <= f.n; ++j) w = fmaf(f.c[j], f.src[j][i * f.stride[j]], w);
    }
    if (compress && i >= cp.cbegin && i < cp.cend) w = compress_one(w, w0, cp, kept);
    out[i] = w;
  }
  if (compress) block_add_count(kept, cp.kept);
}

// Standalone compression epilogue (no mixing): y in place.
__global__ __launch_bounds__(kBlock) void compress_kernel(float* y, const float* ref, long long P,
                                                          CompressParams cp) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    const float r = ref ? ref[i] : 0.0f;
    y[i] = compress_one(y[i], r, cp, kept);
  }
  block_add_count(kept, cp.kept);
}

// ------------------------------------------------------------------------------------------
// TF1 numerics (cfa_mix_tf1_f32): the reference's chain under numpy 2 is fp32 for the first
// subtraction and fp64 after it (eps * wf is an np.float64), so w is carried in double and
// rounded to fp32 once, after the (fp64) compression epilogue. Fan-ins above CFA_MAX_FANIN
// chain passes through an fp64 scratch bucket (FROM64 / TO64).
// ------------------------------------------------------------------------------------------
struct Tf1Fanin {
  const float* local;               // pre-mix local: step-0 input and DPCM reference
  const double* w64;                // running fp64 w of the previous pass (FROM64)
  const float* src[CFA_MAX_FANIN];  // neighbours of this pass
  double a[CFA_MAX_FANIN];          // eps * wf_j
};

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

template <int N, bool FROM64, bool TO64>
__global__ __launch_bounds__(kBlock) void mix_tf1_vec_kernel(void* out, Tf1Fanin f, long long nvec,
                                                              CompressParams cp, int compress) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec;
       i += (long long)gridDim.x * kBlock) {
    f4 x[N];
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = ld4<true>(f.src[k], i);
    const f4 l = ld4<true>(f.local, i);
    double w[4];
    constexpr int j0 = FROM64 ? 0 : 1;
    if constexpr (FROM64) {
#pragma unroll
      for (int c = 0; c < 4; ++c) w[c] = f.w64[4 * i + c];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float d = x[0][c] - l[c];         // fp32 - fp32 (both operands fp32)
        w[c] = (double)l[c] + f.a[0] * (double)d;  // np.float64 * fp32 -> fp64; fp32 + fp64 -> fp64
      }
    }
#pragma unroll
    for (int j = j0; j < N; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) w[c] = w[c] + f.a[j] * ((double)x[j][c] - w[c]);
    if constexpr (TO64) {
      double* o = reinterpret_cast<double*>(out) + 4 * i;
#pragma unroll
      for (int c = 0; c < 4; ++c) o[c] = w[c];
    } else {
      if (compress) {
        const long long e0 = i * 4;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (e0 + c >= cp.cbegin && e0 + c < cp.cend) w[c] = compress_one_d(w[c], l[c], cp, kept);
      }
      const f4 y = {(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
      st4<true>(reinterpret_cast<float*>(out), i, y);
    }
  }
  if (!TO64 && compress) block_add_count(kept, cp.kept);
}

// Scalar TF1 path (misaligned buckets, head and tail pieces).
__global__ __launch_bounds__(kBlock) void mix_tf1_scalar_kernel(void* out, int to64, Tf1Fanin f,
                                                                int n, long long P,
                                                                CompressParams cp, int compress) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    const float l = f.local[i];
    double w;
    int j = 0;
    if (f.w64) {
      w = f.w64[i];
    } else {
      const float d = f.src[0][i] - l;
      w = (double)l + f.a[0] * (double)d;
      j = 1;
    }
    for (; j < n; ++j) w = w + f.a[j] * ((double)f.src[j][i] - w);
    if (to64) {
      reinterpret_cast<double*>(out)[i] = w;
    } else {
      if (compress && i >= cp.cbegin && i < cp.cend) w = compress_one_d(w, l, cp, kept);
      reinterpret_cast<float*>(out)[i] = (float)w;
    }
  }
  if (!to64 && compress) block_add_count(kept, cp.kept);
}

// fp64 buckets (cfa_mix_tf1_f64 / cfa_mewma_tf1_f64): the reference's TF1 arrays as they are
// (fp32 values widened exactly, fp64 values untouched), the same fp64 operations, no rounding.
struct F64Fanin {
  const double* src[CFA_MAX_FANIN + 1];  // [0] = running w (local or previous pass), [1..m]
  double a[CFA_MAX_FANIN + 1];
  double d[CFA_MAX_FANIN + 1];           // SEQUENTIAL_DIV divisors
  int m;
};
// rule: CFA_RULE_SEQUENTIAL  w = w + a*(x - w)
//       CFA_RULE_SEQUENTIAL_DIV  w = w + (a*(x - w))/d
//       CFA_RULE_ACCUMULATE  w = w + a*x
__global__ __launch_bounds__(kBlock) void mix_tf1_f64_kernel(double* out, F64Fanin f, long long P,
                                                             int rule, int step0_f32,
                                                             const double* ref, CompressParams cp,
                                                             int compress) {
  unsigned kept = 0;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    double w = f.src[0][i];
    int j = 1;
    if (step0_f32 && f.m >= 1) {  // both operands fp32 arrays in the reference: fp32 subtraction
      const float d = (float)f.src[1][i] - (float)w;
      w = w + f.a[1] * (double)d;
      j = 2;
    }
    if (rule == CFA_RULE_SEQUENTIAL) {
      for (; j <= f.m; ++j) w = w + f.a[j] * (f.src[j][i] - w);
    } else if (rule == CFA_RULE_SEQUENTIAL_DIV) {
      for (; j <= f.m; ++j) w = w + (f.a[j] * (f.src[j][i] - w)) / f.d[j];
    } else {
      for (; j <= f.m; ++j) w = w + f.a[j] * f.src[j][i];
    }
    if (compress && i >= cp.cbegin && i < cp.cend) w = compress_one_d(w, ref[i], cp, kept);
    out[i] = w;
  }
  if (compress) block_add_count(kept, cp.kept);
}

struct MewmaF64Args {
  double* W;
  double* s[CFA_MAX_FANIN];
  const double* g[CFA_MAX_FANIN];
  long long gstride[CFA_MAX_FANIN];
  int n;
  double rho, one_minus_rho, lr1, lr2;
  long long split;
  int init, filtered, mask;  // mask: CFA_TF1_STATE_F32 | CFA_TF1_GRAD_F32 | CFA_TF1_W_F32
};
// Python-float scalar times an array, in the array's dtype (numpy 2: the scalar is weak).
__device__ __forceinline__ double scale(double c, double x, bool f32) {
  return f32 ? (double)((float)c * (float)x) : c * x;
}
// cfa_ge_2stage.py:331-371 / :593-621 with numpy 2 promotion per operation:
//   s_j = rho*g_j + (1-rho)*s_j (or g_j at init), stored in the state array's dtype;
//   W   = W - lr*(filtered ? s_j : g_j).
// Each product is computed in its array's dtype; a sum or difference is fp32 only when both
// operands are fp32, and W stays fp32 only while every update it receives is fp32.
__global__ __launch_bounds__(kBlock) void mewma_tf1_f64_kernel(MewmaF64Args a, long long P) {
  const bool s32 = a.mask & CFA_TF1_STATE_F32, g32 = a.mask & CFA_TF1_GRAD_F32;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    double W = a.W[i];
    bool w32 = a.mask & CFA_TF1_W_F32;
    const double lr = i < a.split ? a.lr1 : a.lr2;
    for (int j = 0; j < a.n; ++j) {
      const double g = a.g[j][i * a.gstride[j]];
      double s;
      if (a.init) {
        s = g;
      } else {
        const double t1 = scale(a.rho, g, g32);
        const double t2 = scale(a.one_minus_rho, a.s[j][i], s32);
        s = (g32 && s32) ? (double)((float)t1 + (float)t2) : t1 + t2;
      }
      if (s32) s = (double)(float)s;
      a.s[j][i] = s;
      const bool u32 = a.filtered ? s32 : g32;
      const double t = scale(lr, a.filtered ? s : g, u32);
      if (w32 && u32) {
        W = (double)((float)W - (float)t);
      } else {
        W = W - t;
        w32 = false;
      }
    }
    a.W[i] = W;
  }
}

// ------------------------------------------------------------------------------------------
// CFA-GE MEWMA update (TF1/consensus/cfa_ge_2stage.py:593-621, :329-371).
// ------------------------------------------------------------------------------------------
struct MewmaArgs {
  float* W;
  float* s[CFA_MAX_FANIN];
  const float* g[CFA_MAX_FANIN];
  long long gstride[CFA_MAX_FANIN];
  int n;
  float rho, one_minus_rho, lr1, lr2;
  long long split;
  int init, filtered;
};

// Contiguous case: float4 per lane, g and s streamed once each.
__global__ __launch_bounds__(kBlock) void mewma_vec_kernel(MewmaArgs a, long long nvec) {
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec;
       i += (long long)gridDim.x * kBlock) {
    f4 W = ld4<false>(a.W, i);
    const long long e0 = i * 4;
    f4 lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) lr[c] = (e0 + c) < a.split ? a.lr1 : a.lr2;
    for (int j = 0; j < a.n; ++j) {
      const f4 g = ld4<false>(a.g[j], i);
      f4 s;
      if (a.init) {
        s = g;
      } else {
        const f4 s_old = ld4<false>(a.s[j], i);
        s = a.rho * g + a.one_minus_rho * s_old;  // numpy: rho*g + (1-rho)*s
      }
      st4<false>(a.s[j], i, s);
      W = W - lr * (a.filtered ? s : g);
    }
    st4<false>(a.W, i, W);
  }
}

// Generic case: scalar, arbitrary element stride on the gradient buckets.
__global__ __launch_bounds__(kBlock) void mewma_scalar_kernel(MewmaArgs a, long long begin,
                                                              long long P) {
  for (long long i = begin + (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    float W = a.W[i];
    const float lr = i < a.split ? a.lr1 : a.lr2;
    for (int j = 0; j < a.n; ++j) {
      const float g = a.g[j][i * a.gstride[j]];
      float s;
      if (a.init) {
        s = g;
      } else {
        float t1 = a.rho * g;
        float t2 = a.one_minus_rho * a.s[j][i];
        s = t1 + t2;
      }
      a.s[j][i] = s;
      float u = lr * (a.filtered ? s : g);
      W = W - u;
    }
    a.W[i] = W;
  }
}

// ------------------------------------------------------------------------------------------
// Population round: grid.y = device, grid.x = tiles. CSR lists each device's sources.
// ------------------------------------------------------------------------------------------
template <int RULE>
__global__ __launch_bounds__(kBlock) void population_kernel(float* const* out_ptrs,
                                                            const float* const* src_ptrs,
                                                            const int32_t* csr_ptr,
                                                            const int32_t* csr_idx,
                                                            const float* csr_coef,
                                                            long long nvec) {
  const int d = blockIdx.y;
  const int e0 = csr_ptr[d];
  const int e1 = csr_ptr[d + 1];
  float* out = out_ptrs[d];
  constexpr int U = 2;
  constexpr long long kTile = (long long)kBlock * U;
  for (long long t = blockIdx.x; t * kTile < nvec; t += gridDim.x) {
    long long idx[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      idx[u] = t * kTile + (long long)u * kBlock + threadIdx.x;
      ok[u] = idx[u] < nvec;
    }
    f4 w[U];
    const float* s0 = src_ptrs[csr_idx[e0]];
    const float c0 = csr_coef[e0];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      w[u] = ok[u] ? ld4<true>(s0, idx[u]) : f4{0.f, 0.f, 0.f, 0.f};
      if constexpr (RULE == CFA_RULE_LINEAR) w[u] = c0 * w[u];
    }
    for (int e = e0 + 1; e < e1; ++e) {
      const float* s = src_ptrs[csr_idx[e]];
      const float c = csr_coef[e];
      f4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ok[u] ? ld4<true>(s, idx[u]) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (RULE == CFA_RULE_SEQUENTIAL) {
          f4 tt = x[u] - w[u];
          tt = c * tt;
          w[u] = w[u] + tt;
        } else {
          w[u].x = fmaf(c, x[u].x, w[u].x);
          w[u].y = fmaf(c, x[u].y, w[u].y);
          w[u].z = fmaf(c, x[u].z, w[u].z);
          w[u].w = fmaf(c, x[u].w, w[u].w);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (ok[u]) st4<true>(out, idx[u], w[u]);
  }
}

// Scalar tail for the population kernel (elements [begin, P)).
template <int RULE>
__global__ __launch_bounds__(kBlock) void population_tail_kernel(
    float* const* out_ptrs, const float* const* src_ptrs, const int32_t* csr_ptr,
    const int32_t* csr_idx, const float* csr_coef, long long begin, long long P) {
  const int d = blockIdx.y;
  const long long i = begin + threadIdx.x;
  if (i >= P) return;
  const int e0 = csr_ptr[d], e1 = csr_ptr[d + 1];
  float w = src_ptrs[csr_idx[e0]][i];
  if constexpr (RULE == CFA_RULE_LINEAR) w = csr_coef[e0] * w;
  for (int e = e0 + 1; e < e1; ++e) {
    const float x = src_ptrs[csr_idx[e]][i];
    const float c = csr_coef[e];
    if constexpr (RULE == CFA_RULE_SEQUENTIAL) {
      float tt = x - w;
      tt = c * tt;
      w = w + tt;
    } else {
      w = fmaf(c, x, w);
    }
  }
  out_ptrs[d][i] = w;
}

// ------------------------------------------------------------------------------------------
// Sliding-window population pass (cfa_mix_window_f32): nb <= 8 consecutive devices of a ring
// window (hl below, hr above) share their rows, so each row of the window is loaded ONCE per
// element for all nb devices: (nb + hl + hr) reads + nb writes instead of nb * (hl + hr + 2).
// Device b's local row is rows[b + hl]; its neighbours, in the reference window's order
// (g-hl .. g-1, g+1 .. g+hr), are rows[b .. b+hl-1], rows[b+hl+1 .. b+hl+hr].
// ------------------------------------------------------------------------------------------
constexpr int kWinMaxDev = 8;
struct WindowArgs {
  const float* rows[kWinMaxDev + 8];
  float* out[kWinMaxDev];
  float a[kWinMaxDev];  // one coefficient per device, used for each of its steps
  int nb;
};

template <int HL, int HR>
__device__ __forceinline__ f4 window_fold(const f4* r, int b, const WindowArgs& w) {
  f4 acc = r[b + HL];
#pragma unroll
  for (int j = 0; j < HL; ++j) {
    f4 t = r[b + j] - acc;
    t = w.a[b] * t;
    acc = acc + t;
  }
#pragma unroll
  for (int j = 0; j < HR; ++j) {
    f4 t = r[b + HL + 1 + j] - acc;
    t = w.a[b] * t;
    acc = acc + t;
  }
  return acc;
}

template <int HL, int HR, int U, bool SC1>
__global__ __launch_bounds__(kBlock) void window_vec_kernel(WindowArgs w, long long nvec) {
  constexpr int R = kWinMaxDev + HL + HR;
  constexpr long long kTile = (long long)kBlock * U;
  const int nr = w.nb + HL + HR;
  for (long long t = blockIdx.x; t * kTile < nvec; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    f4 r[U][R];
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (k < nr)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long i = base + (long long)u * kBlock;
          if (i < nvec) r[u][k] = ld4<true>(w.rows[k], i);
        }
#pragma unroll
    for (int b = 0; b < kWinMaxDev; ++b)
      if (b < w.nb) {
        // (unused and removed by the compiler when !SC1) write-through streaming store
        const __amdgpu_buffer_rsrc_t o =
            __builtin_amdgcn_make_buffer_rsrc((void*)w.out[b], 0, (unsigned)(nvec * 16), 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long i = base + (long long)u * kBlock;
          if (i < nvec) {
            const f4 y = window_fold<HL, HR>(r[u], b, w);
            if constexpr (SC1)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y), o, (int)(i * 16), 0, kStoreSc1);
            else
              st4<true>(w.out[b], i, y);
          }
        }
      }
  }
}

// Scalar window pass (misaligned rows, the < 4-element tail): runtime hl / hr.
__global__ __launch_bounds__(kBlock) void window_scalar_kernel(WindowArgs w, int hl, int hr,
                                                               long long begin, long long P) {
  for (long long i = begin + (long long)blockIdx.x * kBlock + threadIdx.x; i < P;
       i += (long long)gridDim.x * kBlock) {
    for (int b = 0; b < w.nb; ++b) {
      float acc = w.rows[b + hl][i];
      for (int j = 0; j < hl; ++j) {
        float t = w.rows[b + j][i] - acc;
        t = w.a[b] * t;
        acc = acc + t;
      }
      for (int j = 0; j < hr; ++j) {
        float t = w.rows[b + hl + 1 + j][i] - acc;
        t = w.a[b] * t;
        acc = acc + t;
      }
      w.out[b][i] = acc;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Host-side dispatch.
// ------------------------------------------------------------------------------------------
template <int RULE, int U, bool NT>
static void launch_vec_u(int n, unsigned grid, hipStream_t st, float* out, const Fanin& f,
                         long long nvec) {
#define CFA_CASE(K) \
  case K:           \
    mix_vec_kernel<K, RULE, U, NT><<<grid, kBlock, 0, st>>>(out, f, nvec); \
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
  const int U = t.vec_per_lane > 0 ? norm_vec(t.vec_per_lane) : auto_vec(n);
  const long long tiles = (nvec + (long long)kBlock * U - 1) / ((long long)kBlock * U);
  const unsigned grid = grid_for(tiles, t);
  if (U == 4) {
    if (t.nontemporal) launch_vec_u<RULE, 4, true>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 4, false>(n, grid, st, out, f, nvec);
  } else if (U == 2) {
    if (t.nontemporal) launch_vec_u<RULE, 2, true>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 2, false>(n, grid, st, out, f, nvec);
  } else {
    if (t.nontemporal) launch_vec_u<RULE, 1, true>(n, grid, st, out, f, nvec);
    else launch_vec_u<RULE, 1, false>(n, grid, st, out, f, nvec);
  }
}

static void launch_vec_compress(int n, hipStream_t st, float* out, const Fanin& f, long long nvec,
                                const CompressParams& cp) {
  const unsigned grid = grid_for((nvec + kBlock - 1) / kBlock);
#define CFA_CASE(K) \
  case K:           \
    mix_vec_compress_kernel<K><<<grid, kBlock, 0, st>>>(out, f, nvec, cp); \
    break;
  switch (n) {
    CFA_CASE(0) CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6)
    CFA_CASE(7) CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13)
    CFA_CASE(14) CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
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
    sf.stride[0] = 1;
    for (int j = 0; j < n; ++j) {
      sf.src[j + 1] = nbrs[j] + b;
      sf.stride[j + 1] = 1;
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

// Sequential rule over any fan-in: chunks of CFA_MAX_FANIN; chunk k>0 continues from `out`.
// The compression epilogue is fused into the (single) pass when n <= CFA_MAX_FANIN; wider
// fan-ins run it as a separate pass with the untouched pre-mix `local` as DPCM reference.
static bool needs_ref(int mode) {
  return mode == CFA_COMPRESS_SPARSE_DPCM || mode == CFA_COMPRESS_SPARSE_DPCM_HI;
}
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

template <bool FROM64, bool TO64>
static void launch_tf1_vec(int n, unsigned grid, hipStream_t st, void* out, const Tf1Fanin& f,
                           long long nvec, const CompressParams& cp, int compress) {
#define CFA_CASE(K) \
  case K:           \
    mix_tf1_vec_kernel<K, FROM64, TO64><<<grid, kBlock, 0, st>>>(out, f, nvec, cp, compress); \
    break;
  switch (n) {
    CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6) CFA_CASE(7)
    CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13) CFA_CASE(14)
    CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
}

// One TF1 pass of 1..CFA_MAX_FANIN neighbours over [0, P): `head` scalar elements, a float4
// body of nvec vectors, a scalar tail. out is fp32 (last pass) or the fp64 scratch.
static int tf1_pass(void* out, bool to64, const float* local, const double* w64,
                    const float* const* nbrs, const double* a, int m, size_t P, size_t head,
                    size_t nvec, const CompressParams& cp, int compress, hipStream_t st) {
  auto fanin_at = [&](size_t b) {
    Tf1Fanin f{};
    f.local = local + b;
    f.w64 = w64 ? w64 + b : nullptr;
    for (int j = 0; j < m; ++j) {
      f.src[j] = nbrs[j] + b;
      f.a[j] = a[j];
    }
    return f;
  };
  auto out_at = [&](size_t b) -> void* {
    return to64 ? (void*)((double*)out + b) : (void*)((float*)out + b);
  };
  auto shifted = [&](size_t b) {
    CompressParams c = cp;
    c.cbegin = cp.cbegin - (long long)b;
    c.cend = cp.cend - (long long)b;
    return c;
  };
  if (nvec > 0) {
    const Tf1Fanin f = fanin_at(head);
    const unsigned grid = grid_for(((long long)nvec + kBlock - 1) / kBlock);
    const CompressParams c = shifted(head);
    void* o = out_at(head);
    if (!w64 && !to64) launch_tf1_vec<false, false>(m, grid, st, o, f, (long long)nvec, c, compress);
    else if (!w64 && to64) launch_tf1_vec<false, true>(m, grid, st, o, f, (long long)nvec, c, compress);
    else if (w64 && to64) launch_tf1_vec<true, true>(m, grid, st, o, f, (long long)nvec, c, compress);
    else launch_tf1_vec<true, false>(m, grid, st, o, f, (long long)nvec, c, compress);
    if (int rc = check_launch("mix_tf1_vec")) return rc;
  }
  const size_t tail_begin = head + nvec * 4;
  const size_t pieces[2][2] = {{0, head}, {tail_begin, P}};
  for (auto& pc : pieces) {
    const size_t b = pc[0], e = pc[1];
    if (e <= b) continue;
    const long long len = (long long)(e - b);
    mix_tf1_scalar_kernel<<<grid_for((len + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        out_at(b), to64 ? 1 : 0, fanin_at(b), m, len, shifted(b), compress);
    if (int rc = check_launch("mix_tf1_scalar")) return rc;
  }
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
  cfa_launch_t lc = launch ? *launch : tune();
  if (lc.blocks_per_cu < 0) return fail(CFA_E_INVALID, "blocks_per_cu < 0");
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

extern "C" int cfa_mix_strided_f32(float* out, const float* local, const float* const* nbrs,
                                   const int64_t* nbr_stride, const float* alphas, int n, size_t P,
                                   void* stream) {
  if (n > 0 && (!alphas || !nbr_stride)) return fail(CFA_E_INVALID, "null alphas/strides");
  if (int rc = validate_mix(out, local, nbrs, n, P)) return rc;
  if (P == 0) return CFA_OK;
  bool unit = true;
  for (int j = 0; j < n; ++j) {
    if (nbr_stride[j] < 1) return fail(CFA_E_INVALID, "stride %lld < 1", (long long)nbr_stride[j]);
    unit = unit && nbr_stride[j] == 1;
  }
  if (unit) return cfa_mix_seq_f32(out, local, nbrs, alphas, n, P, stream);
  hipStream_t st = (hipStream_t)stream;
  int done = 0;
  const float* w = local;
  do {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    ScalarFanin sf{};
    sf.src[0] = w;
    sf.stride[0] = 1;
    sf.c[0] = 1.0f;
    for (int j = 0; j < m; ++j) {
      sf.src[j + 1] = nbrs[done + j];
      sf.stride[j + 1] = nbr_stride[done + j];
      sf.c[j + 1] = alphas[done + j];
    }
    sf.n = m;
    CompressParams none{};
    mix_scalar_kernel<<<grid_for(((long long)P + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        out, sf, (long long)P, CFA_RULE_SEQUENTIAL, 0, none);
    if (int rc = check_launch("mix_strided")) return rc;
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
      CFA_HIP_CHECK(hipMemcpyAsync(out, local, P * sizeof(float), hipMemcpyDeviceToDevice, st));
    return cfa_compress_epilogue_f32(out + cbegin, local + cbegin, mode, cend - cbegin,
                                     kept_count, stream);
  }
  return mix_seq_any(out, local, nbrs, alphas, n, P, &cp, st);
}

extern "C" int cfa_mix_tf1_f32(float* out, const float* local, const float* const* nbrs,
                               const double* alphas, int n, size_t P, int mode, size_t cbegin,
                               size_t cend, unsigned long long* kept_count, void* stream) {
  if (n > 0 && !alphas) return fail(CFA_E_INVALID, "null alphas");
  if (mode != CFA_COMPRESS_NONE && !kept_count) return fail(CFA_E_INVALID, "null kept_count");
  // With a counter the epilogue runs (mode 0 keeps, and counts, every element of the range).
  if (cbegin > cend || cend > P) return fail(CFA_E_INVALID, "bad compression range");
  if (int rc = validate_mix(out, local, nbrs, n, P)) return rc;
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  cp.cbegin = (long long)cbegin;
  cp.cend = (long long)cend;
  cp.kept = kept_count;
  const int compress = kept_count ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    // No neighbour: the bucket is the local model (fp32), then the epilogue (cfa_ongraphs.py:218-223).
    if (out != local && P > 0)
      CFA_HIP_CHECK(hipMemcpyAsync(out, local, P * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (!compress) return CFA_OK;
    return cfa_compress_epilogue_f32(out + cbegin, local + cbegin, mode, cend - cbegin, kept_count,
                                     stream);
  }
  if (P == 0) return CFA_OK;
  // Body/head/tail split shared by every pass (fp32 pointers decide it; the fp64 scratch is
  // indexed like the bucket and only needs 8-byte alignment).
  const uintptr_t mis = addr(out) & 15;
  bool same = (addr(local) & 15) == mis;
  for (int j = 0; j < n; ++j) same = same && ((addr(nbrs[j]) & 15) == mis);
  size_t head = P, nvec = 0;
  if (same && (mis & 3) == 0) {
    head = mis ? (16 - mis) / 4 : 0;
    if (head > P) head = P;
    nvec = (P - head) / 4;
  }
  double* scratch = nullptr;
  if (n > CFA_MAX_FANIN)
    CFA_HIP_CHECK(hipMallocAsync((void**)&scratch, P * sizeof(double), st));
  int rc = CFA_OK;
  for (int done = 0; done < n && rc == CFA_OK;) {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    const bool last = done + m == n;
    rc = tf1_pass(last ? (void*)out : (void*)scratch, !last, local, done ? scratch : nullptr,
                  nbrs + done, alphas + done, m, P, head, nvec, cp, last ? compress : 0, st);
    done += m;
  }
  if (scratch) {
    hipError_t e = hipFreeAsync(scratch, st);
    if (rc == CFA_OK && e != hipSuccess) return fail(CFA_E_HIP, "hipFreeAsync: %s", hipGetErrorString(e));
  }
  return rc;
}

namespace {
int fold_f64(double* out, const double* local, const double* const* nbrs, const double* alphas,
             const double* divisors, int n, int rule, int step0_f32, size_t P, int mode,
             size_t cbegin, size_t cend, unsigned long long* kept_count, hipStream_t st) {
  if (n < 0) return fail(CFA_E_INVALID, "negative fan-in %d", n);
  if (n > 0 && (!alphas || !nbrs)) return fail(CFA_E_INVALID, "null alphas/neighbour table");
  if (rule == CFA_RULE_SEQUENTIAL_DIV && n > 0 && !divisors) return fail(CFA_E_INVALID, "null divisors");
  if (rule != CFA_RULE_SEQUENTIAL && rule != CFA_RULE_SEQUENTIAL_DIV && rule != CFA_RULE_ACCUMULATE)
    return fail(CFA_E_INVALID, "rule %d has no fp64 fold", rule);
  if (step0_f32 && rule != CFA_RULE_SEQUENTIAL)
    return fail(CFA_E_INVALID, "step0_f32 applies to the sequential rule only");
  if (mode != CFA_COMPRESS_NONE && !kept_count) return fail(CFA_E_INVALID, "null kept_count");
  if (cbegin > cend || cend > P) return fail(CFA_E_INVALID, "bad compression range");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  if (P == 0) return CFA_OK;
  if (!out || !local) return fail(CFA_E_INVALID, "null out/local bucket");
  for (int j = 0; j < n; ++j) {
    if (!nbrs[j]) return fail(CFA_E_INVALID, "null neighbour bucket %d", j);
    if (nbrs[j] == out) return fail(CFA_E_INVALID, "output aliases neighbour %d", j);
  }
  const int compress = kept_count ? 1 : 0;
  if (compress && out == local && n > CFA_MAX_FANIN && (mode == CFA_COMPRESS_SPARSE_DPCM ||
                                                        mode == CFA_COMPRESS_SPARSE_DPCM_HI))
    return fail(CFA_E_INVALID, "in-place DPCM compression needs fan-in <= %d", CFA_MAX_FANIN);
  cp.cbegin = (long long)cbegin;
  cp.cend = (long long)cend;
  cp.kept = kept_count;
  const unsigned grid = grid_for(((long long)P + kBlock - 1) / kBlock);
  int done = 0;
  const double* w = local;
  do {  // n == 0 runs one pass that copies local (and applies the epilogue)
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    const bool last = done + m == n;
    F64Fanin f{};
    f.src[0] = w;
    f.m = m;
    for (int j = 0; j < m; ++j) {
      f.src[j + 1] = nbrs[done + j];
      f.a[j + 1] = alphas[done + j];
      f.d[j + 1] = divisors ? divisors[done + j] : 1.0;
    }
    mix_tf1_f64_kernel<<<grid, kBlock, 0, st>>>(out, f, (long long)P, rule,
                                                done == 0 ? step0_f32 : 0, local, cp,
                                                last ? compress : 0);
    if (int rc = check_launch("fold_f64")) return rc;
    done += m;
    w = out;
  } while (done < n);
  return CFA_OK;
}
}  // namespace

extern "C" int cfa_mix_tf1_f64(double* out, const double* local, const double* const* nbrs,
                               const double* alphas, int n, int step0_f32, size_t P, int mode,
                               size_t cbegin, size_t cend, unsigned long long* kept_count,
                               void* stream) {
  return fold_f64(out, local, nbrs, alphas, nullptr, n, CFA_RULE_SEQUENTIAL, step0_f32, P, mode,
                  cbegin, cend, kept_count, (hipStream_t)stream);
}

extern "C" int cfa_fold_f64(double* out, const double* local, const double* const* nbrs,
                            const double* alphas, const double* divisors, int n, int rule,
                            size_t P, void* stream) {
  return fold_f64(out, local, nbrs, alphas, divisors, n, rule, 0, P, CFA_COMPRESS_NONE, 0, 0,
                  nullptr, (hipStream_t)stream);
}

extern "C" int cfa_mewma_tf1_f64(double* W, double* const* s, const double* const* g,
                                 const int64_t* g_stride, int n, double rho, double lr1,
                                 double lr2, size_t lr_split, int init, int use_filtered,
                                 int f32_mask, size_t P, void* stream) {
  if (n < 0) return fail(CFA_E_INVALID, "negative fan-in %d", n);
  if (n > 0 && (!s || !g)) return fail(CFA_E_INVALID, "null state/gradient table");
  if (f32_mask & ~(CFA_TF1_STATE_F32 | CFA_TF1_GRAD_F32 | CFA_TF1_W_F32))
    return fail(CFA_E_INVALID, "unknown dtype mask bits 0x%x", f32_mask);
  if (P == 0 || n == 0) return CFA_OK;
  if (!W) return fail(CFA_E_INVALID, "null W");
  hipStream_t st = (hipStream_t)stream;
  for (int done = 0; done < n;) {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    MewmaF64Args a{};
    a.W = W;
    a.n = m;
    for (int j = 0; j < m; ++j) {
      if (!s[done + j] || !g[done + j]) return fail(CFA_E_INVALID, "null state/gradient %d", done + j);
      const long long gs = g_stride ? (long long)g_stride[done + j] : 1;
      if (gs < 1) return fail(CFA_E_INVALID, "gradient stride %lld < 1", gs);
      a.s[j] = s[done + j];
      a.g[j] = g[done + j];
      a.gstride[j] = gs;
    }
    a.rho = rho;
    a.one_minus_rho = 1.0 - rho;  // Python: (1 - self.mewma)
    a.lr1 = lr1;
    a.lr2 = lr2;
    a.split = (long long)lr_split;
    a.init = init;
    a.filtered = use_filtered;
    a.mask = f32_mask;
    mewma_tf1_f64_kernel<<<grid_for(((long long)P + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        a, (long long)P);
    if (int rc = check_launch("mewma_tf1_f64")) return rc;
    done += m;
  }
  return CFA_OK;
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
  compress_kernel<<<grid_for(((long long)P + kBlock - 1) / kBlock), kBlock, 0, st>>>(
      y, ref, (long long)P, cp);
  return check_launch("compress");
}

extern "C" int cfa_mewma_update_f32(float* W, float* const* s, const float* const* g,
                                    const int64_t* g_stride, int n, double rho, float lr1,
                                    float lr2, size_t lr_split, int init, int use_filtered,
                                    size_t P, void* stream) {
  if (n < 0) return fail(CFA_E_INVALID, "negative fan-in %d", n);
  if (P == 0 || n == 0) return CFA_OK;
  if (!W || !s || !g) return fail(CFA_E_INVALID, "null W/s/g");
  hipStream_t st = (hipStream_t)stream;
  for (int done = 0; done < n;) {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    MewmaArgs a{};
    a.W = W;
    a.n = m;
    a.rho = (float)rho;
    a.one_minus_rho = (float)(1.0 - rho);
    a.lr1 = lr1;
    a.lr2 = lr2;
    a.split = (long long)lr_split;
    a.init = init;
    a.filtered = use_filtered;
    bool vec = (addr(W) & 15) == 0;
    for (int j = 0; j < m; ++j) {
      if (!s[done + j] || !g[done + j]) return fail(CFA_E_INVALID, "null s/g bucket %d", done + j);
      a.s[j] = s[done + j];
      a.g[j] = g[done + j];
      a.gstride[j] = g_stride ? g_stride[done + j] : 1;
      if (a.gstride[j] < 1) return fail(CFA_E_INVALID, "gradient stride < 1");
      vec = vec && a.gstride[j] == 1 && (addr(a.s[j]) & 15) == 0 && (addr(a.g[j]) & 15) == 0;
    }
    long long begin = 0;
    if (vec) {
      const long long nvec = (long long)P / 4;
      if (nvec > 0) {
        mewma_vec_kernel<<<grid_for((nvec + kBlock - 1) / kBlock), kBlock, 0, st>>>(a, nvec);
        if (int rc = check_launch("mewma_vec")) return rc;
      }
      begin = nvec * 4;
    }
    if (begin < (long long)P) {
      mewma_scalar_kernel<<<grid_for(((long long)P - begin + kBlock - 1) / kBlock), kBlock, 0,
                            st>>>(a, begin, (long long)P);
      if (int rc = check_launch("mewma_scalar")) return rc;
    }
    done += m;
  }
  return CFA_OK;
}

namespace {
struct WindowTune {
  int vec, sc1, blocks_per_cu;
};
static WindowTune window_tune() {  // env overrides for tools/tune_window.py; results identical
  WindowTune t{1, 0, 6};  // tools/tune_window.py, profiles/r01_tune_window.jsonl
  if (const char* e = getenv("CFA_WINDOW_VEC")) t.vec = atoi(e) == 1 ? 1 : 2;
  if (const char* e = getenv("CFA_WINDOW_SC1")) t.sc1 = atoi(e) ? 1 : 0;
  if (const char* e = getenv("CFA_WINDOW_BLOCKS_PER_CU")) t.blocks_per_cu = atoi(e) > 0 ? atoi(e) : 2;
  return t;
}
template <int HL, int HR>
void launch_window(const WindowArgs& w, long long nvec, hipStream_t st) {
  const WindowTune t = window_tune();
  const cfa_launch_t lc{t.blocks_per_cu, t.vec, 1};
  // chunks of at most kMaxChunkVec float4: 32-bit buffer offsets of the streaming store
  for (long long done = 0; done < nvec; done += kMaxChunkVec) {
    const long long m = (nvec - done) < kMaxChunkVec ? (nvec - done) : kMaxChunkVec;
    WindowArgs c = w;
    for (int k = 0; k < w.nb + HL + HR; ++k) c.rows[k] = w.rows[k] + done * 4;
    for (int b = 0; b < w.nb; ++b) c.out[b] = w.out[b] + done * 4;
    const long long tiles = (m + (long long)kBlock * t.vec - 1) / ((long long)kBlock * t.vec);
    const unsigned grid = grid_for(tiles, lc);
    if (t.vec == 1) {
      if (t.sc1) window_vec_kernel<HL, HR, 1, true><<<grid, kBlock, 0, st>>>(c, m);
      else window_vec_kernel<HL, HR, 1, false><<<grid, kBlock, 0, st>>>(c, m);
    } else {
      if (t.sc1) window_vec_kernel<HL, HR, 2, true><<<grid, kBlock, 0, st>>>(c, m);
      else window_vec_kernel<HL, HR, 2, false><<<grid, kBlock, 0, st>>>(c, m);
    }
  }
}
using WindowLaunch = void (*)(const WindowArgs&, long long, hipStream_t);
#define CFA_W(L, R) &launch_window<L, R>
const WindowLaunch kWindowLaunch[5][5] = {
    {CFA_W(0, 0), CFA_W(0, 1), CFA_W(0, 2), CFA_W(0, 3), CFA_W(0, 4)},
    {CFA_W(1, 0), CFA_W(1, 1), CFA_W(1, 2), CFA_W(1, 3), CFA_W(1, 4)},
    {CFA_W(2, 0), CFA_W(2, 1), CFA_W(2, 2), CFA_W(2, 3), CFA_W(2, 4)},
    {CFA_W(3, 0), CFA_W(3, 1), CFA_W(3, 2), CFA_W(3, 3), CFA_W(3, 4)},
    {CFA_W(4, 0), CFA_W(4, 1), CFA_W(4, 2), CFA_W(4, 3), CFA_W(4, 4)}};
#undef CFA_W
}  // namespace

extern "C" int cfa_mix_window_f32(float* const* out, const float* const* rows, const float* alphas,
                                  int nb, int hl, int hr, size_t P, void* stream) {
  if (nb < 1 || nb > kWinMaxDev) return fail(CFA_E_INVALID, "nb %d outside 1..%d", nb, kWinMaxDev);
  if (hl < 0 || hr < 0 || hl > 4 || hr > 4) return fail(CFA_E_INVALID, "window %d/%d outside 0..4", hl, hr);
  if (!out || !rows || !alphas) return fail(CFA_E_INVALID, "null table");
  if (P == 0) return CFA_OK;
  WindowArgs w{};
  w.nb = nb;
  const int nr = nb + hl + hr;
  bool aligned = true;
  for (int k = 0; k < nr; ++k) {
    if (!rows[k]) return fail(CFA_E_INVALID, "null row %d", k);
    w.rows[k] = rows[k];
    aligned = aligned && (addr(rows[k]) & 15) == 0;
  }
  for (int b = 0; b < nb; ++b) {
    if (!out[b]) return fail(CFA_E_INVALID, "null output %d", b);
    for (int k = 0; k < nr; ++k)
      if (out[b] == rows[k]) return fail(CFA_E_INVALID, "output %d aliases row %d", b, k);
    w.out[b] = out[b];
    aligned = aligned && (addr(out[b]) & 15) == 0;
    w.a[b] = alphas[b];
  }
  hipStream_t st = (hipStream_t)stream;
  const long long nvec = aligned ? (long long)(P / 4) : 0;
  if (nvec > 0) {
    kWindowLaunch[hl][hr](w, nvec, st);
    if (int rc = check_launch("window_vec")) return rc;
  }
  const long long begin = nvec * 4;
  if (begin < (long long)P) {
    const long long len = (long long)P - begin;
    window_scalar_kernel<<<grid_for((len + kBlock - 1) / kBlock), kBlock, 0, st>>>(w, hl, hr, begin, (long long)P);
    if (int rc = check_launch("window_scalar")) return rc;
  }
  return CFA_OK;
}

extern "C" int cfa_mix_population_f32(float* const* out_ptrs, const float* const* src_ptrs,
                                      const int32_t* csr_ptr, const int32_t* csr_idx,
                                      const float* csr_coef, int D, int rule, size_t P,
                                      void* stream) {
  if (D < 0) return fail(CFA_E_INVALID, "negative device count");
  if (rule != CFA_RULE_SEQUENTIAL && rule != CFA_RULE_LINEAR)
    return fail(CFA_E_INVALID, "unknown rule %d", rule);
  if (D == 0 || P == 0) return CFA_OK;
  if (!out_ptrs || !src_ptrs || !csr_ptr || !csr_idx || !csr_coef)
    return fail(CFA_E_INVALID, "null population table");
  if (D > 65535) return fail(CFA_E_INVALID, "D=%d exceeds grid.y limit", D);
  hipStream_t st = (hipStream_t)stream;
  // Buckets in a population are expected 16-byte aligned (allocator contract, checked by the
  // host layer); the body runs on float4, the <4-element tail on the scalar kernel.
  const long long nvec = (long long)P / 4;
  if (nvec > 0) {
    const long long tiles = (nvec + 2LL * kBlock - 1) / (2LL * kBlock);
    long long gx = tiles;
    const long long cap = ((long long)device_cus() * 8 + D - 1) / D;
    if (gx > cap) gx = cap < 1 ? 1 : cap;
    dim3 grid((unsigned)gx, (unsigned)D);
    if (rule == CFA_RULE_SEQUENTIAL)
      population_kernel<CFA_RULE_SEQUENTIAL><<<grid, kBlock, 0, st>>>(out_ptrs, src_ptrs, csr_ptr,
                                                                      csr_idx, csr_coef, nvec);
    else
      population_kernel<CFA_RULE_LINEAR><<<grid, kBlock, 0, st>>>(out_ptrs, src_ptrs, csr_ptr,
                                                                  csr_idx, csr_coef, nvec);
    if (int rc = check_launch("population")) return rc;
  }
  const long long begin = nvec * 4;
  if (begin < (long long)P) {
    dim3 grid(1, (unsigned)D);
    if (rule == CFA_RULE_SEQUENTIAL)
      population_tail_kernel<CFA_RULE_SEQUENTIAL><<<grid, 64, 0, st>>>(
          out_ptrs, src_ptrs, csr_ptr, csr_idx, csr_coef, begin, (long long)P);
    else
      population_tail_kernel<CFA_RULE_LINEAR><<<grid, 64, 0, st>>>(
          out_ptrs, src_ptrs, csr_ptr, csr_idx, csr_coef, begin, (long long)P);
    if (int rc = check_launch("population_tail")) return rc;
  }
  return CFA_OK;
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

// Write-batching experiment: each wave folds B tiles (loads of all 9 streams per tile), keeps
// the B outputs in registers, then stores them in one burst. SOFT: after each batch's reads, the
// workgroup waits (bounded spin, never needed for correctness) until every workgroup has
// finished its reads of that batch, so the chip's write bursts line up in time.
namespace {
__device__ unsigned int g_batch_arrivals;
__global__ void reset_arrivals_kernel() { g_batch_arrivals = 0; }

template <int B, bool SOFT>
__global__ __launch_bounds__(kBlock) void mix8_batch_kernel(float* out, Fanin f, long long nvec,
                                                            int spin_limit) {
  constexpr int N = 8, U = 4;
  __shared__ f4 ybuf[B][U][kBlock];  // thread-private slots: no LDS synchronisation needed
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, (unsigned)(nvec * 16), 0x00020000);
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec / kTile;
  const long long G = gridDim.x;
  unsigned phase = 0;
  for (long long t0 = blockIdx.x; t0 < full; t0 += G * B, ++phase) {
#pragma unroll 1
    for (int b = 0; b < B; ++b) {
      const long long t = t0 + b * G;
      if (t < full) {
        const long long base = t * kTile + threadIdx.x;
        f4 v[U][N + 1];
#pragma unroll
        for (int k = 0; k <= N; ++k)
#pragma unroll
          for (int u = 0; u < U; ++u) v[u][k] = ld4<true>(f.src[k], base + (long long)u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) ybuf[b][u][threadIdx.x] = fold<N, CFA_RULE_SEQUENTIAL>(v[u], f);
      }
    }
    if constexpr (SOFT) {
      __syncthreads();
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(&g_batch_arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (phase + 1) * (unsigned)G;
        for (int i = 0; i < spin_limit; ++i) {
          if (__hip_atomic_load(&g_batch_arrivals, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const long long t = t0 + b * G;
      if (t < full) {
        const long long base = t * kTile + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, ybuf[b][u][threadIdx.x]), w,
                                                 (int)((base + (long long)u * kBlock) * 16), 0, kStoreSc1);
      }
    }
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int cfa_experimental_mix8_batch(
    float* out, const float* local, const float* const* nbrs, const float* alphas, size_t P,
    int batch, int soft, int spin_limit, int blocks_per_cu, void* stream) {
  if (P % 4096 || P * 4 > 0xffffffffull) return fail(CFA_E_INVALID, "experiment needs P %% 4096 == 0, < 4 GiB");
  if (spin_limit < 0 || spin_limit > 100000) return fail(CFA_E_INVALID, "spin_limit out of range");
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
  if (soft) {
    reset_arrivals_kernel<<<1, 1, 0, st>>>();
    if (int rc = check_launch("reset_arrivals")) return rc;
  }
#define CFA_B(BB)                                                                              \
  if (batch == BB) {                                                                           \
    if (soft) mix8_batch_kernel<BB, true><<<grid, kBlock, 0, st>>>(out, f, nvec, spin_limit);  \
    else mix8_batch_kernel<BB, false><<<grid, kBlock, 0, st>>>(out, f, nvec, spin_limit);      \
    return check_launch("mix8_batch");                                                         \
  }
  CFA_B(1) CFA_B(2) CFA_B(4)
#undef CFA_B
  return fail(CFA_E_INVALID, "batch must be 1, 2 or 4");
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
