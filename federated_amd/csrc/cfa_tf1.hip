// cfa_tf1.hip — the reference's TF1 numerics under numpy 2 (fp32 first subtraction, fp64 after),
// on fp32 buckets rounded once (cfa_mix_tf1_f32) or on fp64 buckets unrounded (cfa_mix_tf1_f64,
// cfa_fold_f64, cfa_mewma_tf1_f64): TF1/consensus/cfa.py:69-76, cfa_ongraphs.py:112-119 and
// 225-273, cfa_ge_2stage.py:76-83, 331-371, 593-621; the fp64 server-side folds of
// FL_over_MQTT/PS_server.py:130-133, learner_consensus.py:151-152,
// federated_sample_CNN_CFA_FA.py:86-89, 130-133, 280-283.
#include <utility>

#include "cfa_internal.h"

namespace {

// ------------------------------------------------------------------------------------------
// TF1 numerics (cfa_mix_tf1_f32): the reference's chain under numpy 2 is fp32 for the first
// subtraction and fp64 after it (eps * wf is an np.float64), so w is carried in double and
// rounded to fp32 once, after the (fp64) compression epilogue. Fan-ins above CFA_MAX_FANIN
// chain passes through an fp64 scratch bucket (FROM64 / kOutScratch64); cfa_mix_tf1_wide_f32
// writes the unrounded fp64 result instead (and chains its passes in that output).
// ------------------------------------------------------------------------------------------
typedef double d2 __attribute__((ext_vector_type(2)));

struct Tf1Fanin {
  const float* local;               // pre-mix local: step-0 input and DPCM reference
  const double* w64;                // running fp64 w of the previous pass (FROM64)
  const float* src[CFA_MAX_FANIN];  // neighbours of this pass
  double a[CFA_MAX_FANIN];          // eps * wf_j
};

// Output of a TF1 pass: the fp32 result (epilogue, one rounding), the fp64 scratch of a chained
// pass (no epilogue), or the unrounded fp64 result (epilogue in fp64, no rounding).
enum { kOutF32 = 0, kOutScratch64 = 1, kOutF64 = 2 };

// Vector width of the TF1 kernel: float4 per lane for the fp32 output (16-B loads, 16-B stores);
// float2 for the fp64 outputs, so that each lane's result is ONE 16-byte store and a wave's store
// instruction covers 1 KiB contiguously. (With float4 per lane the four fp64 results are two
// 16-B stores at a 32-B lane stride: each store instruction half-fills 16 lines and the other
// half follows in the next instruction.)
template <int OUT>
struct Tf1Vec {
  static constexpr int W = OUT == kOutF32 ? 4 : 2;
  typedef float type __attribute__((ext_vector_type(W)));
};

// One vector of the TF1 chain: x = the N neighbour vectors, l = the local vector, w64 = the
// previous pass's running fp64 w (FROM64), i = the vector's index. Epilogue, rounding and store.
template <int N, bool FROM64, int OUT, typename V = typename Tf1Vec<OUT>::type>
__device__ __forceinline__ void tf1_vec(void* out, const Sc1Out& o, const Tf1Fanin& f, const V (&x)[N],
                                        const V& l, const double* w64, long long i, const CompressParams& cp,
                                        int compress, unsigned& kept) {
  constexpr int W = Tf1Vec<OUT>::W;
  double w[W];
  constexpr int j0 = FROM64 ? 0 : 1;
  if constexpr (FROM64) {
#pragma unroll
    for (int c = 0; c < W; ++c) w[c] = w64[c];
  } else {
#pragma unroll
    for (int c = 0; c < W; ++c) {
      const float d = x[0][c] - l[c];            // fp32 - fp32 (both operands fp32)
      w[c] = (double)l[c] + f.a[0] * (double)d;  // np.float64 * fp32 -> fp64; fp32 + fp64 -> fp64
    }
  }
#pragma unroll
  for (int j = j0; j < N; ++j)
#pragma unroll
    for (int c = 0; c < W; ++c) w[c] = w[c] + f.a[j] * ((double)x[j][c] - w[c]);
  if (OUT != kOutScratch64 && compress) {
    const long long e0 = i * W;
#pragma unroll
    for (int c = 0; c < W; ++c)
      if (e0 + c >= cp.cbegin && e0 + c < cp.cend) w[c] = compress_one_d(w[c], l[c], cp, kept);
  }
  if constexpr (OUT == kOutF32) {
    const f4 y = {(float)w[0], (float)w[1], (float)w[2], (float)w[3]};
    st16_sc1(o, i, y);
  } else {  // fp64 out: one plain 16-B store per lane (sc1 halves measured 17% slower in round 2);
            // mix_tf1_impl sends an fp64 output whose body is not 16-B aligned to the scalar kernel
    const d2 y = {w[0], w[1]};
    reinterpret_cast<d2*>(out)[i] = y;
  }
}

// Full tiles of kBlock * U vectors per block (grid-stride over tiles, every load of a tile issued
// before its first use, nontemporal loads), the partial last tile by the block that owns it with
// per-vector guards: the headline mix's skeleton (round 4). nvec counts vectors of Tf1Vec<OUT>::W
// elements.
template <int N, bool FROM64, int OUT, int U>
__global__ __launch_bounds__(kBlock) void mix_tf1_vec_kernel(void* out, Tf1Fanin f, long long nvec,
                                                              CompressParams cp, int compress) {
  using V = typename Tf1Vec<OUT>::type;
  constexpr int W = Tf1Vec<OUT>::W;
  constexpr long long kTile = (long long)kBlock * U;
  unsigned kept = 0;
  const Sc1Out o = sc1_out(out, nvec * 16);  // used by the fp32 output only (16-B vectors)
  const long long full = nvec / kTile;
  auto ld = [](const float* p, long long i) { return __builtin_nontemporal_load(reinterpret_cast<const V*>(p) + i); };
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    V x[U][N], l[U];
#pragma unroll
    for (int k = 0; k < N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) x[u][k] = ld(f.src[k], base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) l[u] = ld(f.local, base + (long long)u * kBlock);
    double w64[U][W];
    if constexpr (FROM64) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < W; ++c) w64[u][c] = f.w64[W * (base + (long long)u * kBlock) + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      tf1_vec<N, FROM64, OUT>(out, o, f, x[u], l[u], w64[u], base + (long long)u * kBlock, cp, compress, kept);
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec; i += kBlock) {
      V x[N];
#pragma unroll
      for (int k = 0; k < N; ++k) x[k] = ld(f.src[k], i);
      const V l = ld(f.local, i);
      double w64[W];
      if constexpr (FROM64) {
#pragma unroll
        for (int c = 0; c < W; ++c) w64[c] = f.w64[W * i + c];
      }
      tf1_vec<N, FROM64, OUT>(out, o, f, x, l, w64, i, cp, compress, kept);
    }
  }
  if (OUT != kOutScratch64 && compress) block_add_count(kept, cp.kept);
}

// Scalar TF1 path (misaligned buckets, head and tail pieces).
__global__ __launch_bounds__(kBlock) void mix_tf1_scalar_kernel(void* out, int out_mode, Tf1Fanin f,
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
    if (out_mode != kOutScratch64 && compress && i >= cp.cbegin && i < cp.cend)
      w = compress_one_d(w, l, cp, kept);
    if (out_mode == kOutF32)
      reinterpret_cast<float*>(out)[i] = (float)w;
    else
      reinterpret_cast<double*>(out)[i] = w;
  }
  if (out_mode != kOutScratch64 && compress) block_add_count(kept, cp.kept);
}

// fp64 buckets (cfa_mix_tf1_f64 / cfa_mewma_tf1_f64): the reference's TF1 arrays as they are
// (fp32 values widened exactly, fp64 values untouched), the same fp64 operations, no rounding.
struct F64Fanin {
  const double* src[CFA_MAX_FANIN + 1];  // [0] = running w (local or previous pass), [1..m]
  double a[CFA_MAX_FANIN + 1];
  double d[CFA_MAX_FANIN + 1];           // SEQUENTIAL_DIV divisors
  double r[CFA_MAX_FANIN + 1];           // RN(1 / d[j]) for ddiv_rn
  int m;
  int fast_div;                          // every d[j] in [2^-20, 2^20]
};

// Correctly rounded fp64 a / b (Markstein): q = RN(a * rb) with rb = RN(1/b) is within 1 ulp,
// the remainder a - b q is exact (one fma), and RN(q + r * rb) is the correctly rounded quotient
// when nothing under- or overflows; |a| in [2^-900, 2^900] and b in [2^-20, 2^20] guarantee
// that, everything else takes the IEEE division. (The fp32 fold's one-multiply form, div_rd in
// cfa_internal.h, needs a format twice as wide; fp64 has none on the GPU.)
__device__ __forceinline__ double ddiv_rn(double a, double b, double rb, bool fast) {
  const double aa = __builtin_fabs(a);
  if (fast && aa >= 0x1p-900 && aa <= 0x1p900) {
    const double q = a * rb;
    const double r = __builtin_fma(-q, b, a);
    return __builtin_fma(r, rb, q);
  }
  return a / b;
}
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

// Vector form of mix_tf1_f64_kernel for 16-byte-aligned buckets: each lane moves two doubles per
// bucket per vector, U vectors per tile, every load of a tile issued before its first use, the
// fan-in N and the rule at compile time (the runtime loop above serialises its loads). The
// headline mix's skeleton (round 4, tools/probe/lowrow_sweep.py, profiles/r04_lowrow_sweep.jsonl):
// full tiles walked grid-stride with no per-vector guards, the partial tail done by one
// workgroup, and the output through the sc1 write-through buffer store (Sc1Out) at two
// workgroups per CU: the divisor fold at n = 4 went from 0.734 to 0.815 of peak on the same
// buffers (a nontemporal store at one vector per lane: 0.789).
template <int N, int RULE, bool STEP0F32>
__device__ __forceinline__ d2 fold_d2(const d2 (&v)[N + 1], const F64Fanin& f, long long idx, const double* ref,
                                      const CompressParams& cp, int compress, unsigned& kept) {
  d2 y;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    double w = v[0][c];
    int j = 1;
    if constexpr (STEP0F32) {  // both operands fp32 arrays in the reference: fp32 subtraction
      const float d = (float)v[1][c] - (float)w;
      w = w + f.a[1] * (double)d;
      j = 2;
    }
#pragma unroll
    for (int k = 1; k <= N; ++k) {
      if (k < j) continue;
      if constexpr (RULE == CFA_RULE_SEQUENTIAL) w = w + f.a[k] * (v[k][c] - w);
      else if constexpr (RULE == CFA_RULE_SEQUENTIAL_DIV)
        w = w + ddiv_rn(f.a[k] * (v[k][c] - w), f.d[k], f.r[k], f.fast_div);
      else w = w + f.a[k] * v[k][c];
    }
    if (compress) {
      const long long e = 2 * idx + c;
      if (e >= cp.cbegin && e < cp.cend) w = compress_one_d(w, ref[e], cp, kept);
    }
    y[c] = w;
  }
  return y;
}

template <int N, int RULE, bool STEP0F32>
__global__ __launch_bounds__(kBlock) void fold_f64_vec_kernel(double* out, F64Fanin f, long long nvec2,
                                                               const double* ref, CompressParams cp,
                                                               int compress) {
  constexpr int U = 2;
  constexpr long long kTile = (long long)kBlock * U;
  const long long full = nvec2 / kTile;
  const Sc1Out o = sc1_out(out, nvec2 * 16);
  unsigned kept = 0;
  for (long long t = blockIdx.x; t < full; t += gridDim.x) {
    const long long base = t * kTile + threadIdx.x;
    d2 v[U][N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u][k] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(f.src[k]) + base + (long long)u * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + (long long)u * kBlock;
      st16_sc1(o, i, fold_d2<N, RULE, STEP0F32>(v[u], f, i, ref, cp, compress, kept));
    }
  }
  if (blockIdx.x == (unsigned)(full % gridDim.x)) {
    for (long long i = full * kTile + threadIdx.x; i < nvec2; i += kBlock) {
      d2 v[N + 1];
#pragma unroll
      for (int k = 0; k <= N; ++k) v[k] = reinterpret_cast<const d2*>(f.src[k])[i];
      st16_sc1(o, i, fold_d2<N, RULE, STEP0F32>(v, f, i, ref, cp, compress, kept));
    }
  }
  if (compress) block_add_count(kept, cp.kept);
}

template <int RULE, bool STEP0F32>
static void launch_fold_vec(int m, unsigned grid, hipStream_t st, double* out, const F64Fanin& f,
                            long long nvec2, const double* ref, const CompressParams& cp, int compress) {
#define CFA_CASE(K) \
  case K:           \
    fold_f64_vec_kernel<K, RULE, STEP0F32><<<grid, kBlock, 0, st>>>(out, f, nvec2, ref, cp, compress); \
    break;
  switch (m) {
    CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6) CFA_CASE(7)
    CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13) CFA_CASE(14)
    CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
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

// Vector form for unit-stride, 16-byte-aligned buckets: two doubles per lane, the fan-in N at
// compile time so that every W / g / s load is issued before the first update.
// ANY32 = false is the all-fp64 case (mask 0, what the TF1 drivers hold after loadmat / np.zeros):
// the dtype flags are then compile-time false and the per-product fp32 selects disappear.
template <int N, bool ANY32>
__global__ __launch_bounds__(kBlock) void mewma_tf1_f64_vec_kernel(MewmaF64Args a, long long nvec2) {
  const bool s32 = ANY32 && (a.mask & CFA_TF1_STATE_F32), g32 = ANY32 && (a.mask & CFA_TF1_GRAD_F32);
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec2;
       i += (long long)gridDim.x * kBlock) {
    d2 Wv = __builtin_nontemporal_load(reinterpret_cast<const d2*>(a.W) + i);
    d2 g[N], so[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      g[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(a.g[j]) + i);
      if (!a.init) so[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(a.s[j]) + i);
    }
    d2 sn[N];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      double W = Wv[c];
      bool w32 = ANY32 && (a.mask & CFA_TF1_W_F32);
      const double lr = 2 * i + c < a.split ? a.lr1 : a.lr2;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double sv;
        if (a.init) {
          sv = g[j][c];
        } else {
          const double t1 = scale(a.rho, g[j][c], g32);
          const double t2 = scale(a.one_minus_rho, so[j][c], s32);
          sv = (g32 && s32) ? (double)((float)t1 + (float)t2) : t1 + t2;
        }
        if (s32) sv = (double)(float)sv;
        sn[j][c] = sv;
        const bool u32 = a.filtered ? s32 : g32;
        const double t = scale(lr, a.filtered ? sv : g[j][c], u32);
        if (w32 && u32) {
          W = (double)((float)W - (float)t);
        } else {
          W = W - t;
          w32 = false;
        }
      }
      Wv[c] = W;
    }
    // nontemporal here: the default policy measured 6% slower for the fp64 form (unlike fp32),
    // and two vectors per stream per lane were neutral
#pragma unroll
    for (int j = 0; j < N; ++j) __builtin_nontemporal_store(sn[j], reinterpret_cast<d2*>(a.s[j]) + i);
    __builtin_nontemporal_store(Wv, reinterpret_cast<d2*>(a.W) + i);
  }
}

template <int... Ns>
static void launch_mewma_f64_vec(int m, unsigned grid, hipStream_t st, const MewmaF64Args& a, long long nvec2,
                                 std::integer_sequence<int, Ns...>) {
  if (a.mask)
    ((m == Ns + 1 ? (void)(mewma_tf1_f64_vec_kernel<Ns + 1, true><<<grid, kBlock, 0, st>>>(a, nvec2)) : (void)0), ...);
  else
    ((m == Ns + 1 ? (void)(mewma_tf1_f64_vec_kernel<Ns + 1, false><<<grid, kBlock, 0, st>>>(a, nvec2)) : (void)0),
     ...);
}

template <bool FROM64, int OUT, int U>
static void launch_tf1_vec_u(int n, unsigned grid, hipStream_t st, void* out, const Tf1Fanin& f,
                             long long nvec, const CompressParams& cp, int compress) {
#define CFA_CASE(K) \
  case K:           \
    mix_tf1_vec_kernel<K, FROM64, OUT, U><<<grid, kBlock, 0, st>>>(out, f, nvec, cp, compress); \
    break;
  switch (n) {
    CFA_CASE(1) CFA_CASE(2) CFA_CASE(3) CFA_CASE(4) CFA_CASE(5) CFA_CASE(6) CFA_CASE(7)
    CFA_CASE(8) CFA_CASE(9) CFA_CASE(10) CFA_CASE(11) CFA_CASE(12) CFA_CASE(13) CFA_CASE(14)
    CFA_CASE(15) CFA_CASE(16)
    default: break;
  }
#undef CFA_CASE
}

// Launch shape of the TF1 vector kernel: the library default or an explicit CFA_VEC_PER_LANE /
// CFA_BLOCKS_PER_CU. Default (round 4, tools/kernel_rooflines.py A/B, two alternated rounds on one
// box, profiles/r04_tf1_ab_rooflines.jsonl): fp32 out two float4 per lane at two workgroups per CU
// (0.782 / 0.783 of peak at 25M, n = 8, against 0.757 / 0.755 for the one-vector grid-stride
// kernel before; one float4: 0.743, four: 0.757); fp64 out four float2 at one workgroup per CU
// (profiles/r04_tf1b_ab_rooflines.jsonl: 0.781 / 0.781 against 0.754 / 0.755 for four float4,
// whose fp64 results left as two 16-B stores at a 32-B lane stride; float2 with two: 0.759 / 0.753,
// one: 0.701 / 0.711; two workgroups per CU with four: 0.755 / 0.757, with two: 0.719 / 0.730).
template <bool FROM64, int OUT>
static void launch_tf1_vec(int n, hipStream_t st, void* out, const Tf1Fanin& f, long long nvec,
                           const CompressParams& cp, int compress) {
  const cfa_launch_t& t = tune();
  const int U = t.vec_per_lane > 0 ? norm_vec(t.vec_per_lane) : (OUT == kOutF32 ? 2 : 4);
  nvec *= 4 / Tf1Vec<OUT>::W;  // the caller counts float4; the fp64 outputs run float2 vectors
  const long long tiles = (nvec + (long long)kBlock * U - 1) / ((long long)kBlock * U);
  const unsigned grid = OUT == kOutF64 ? grid_for_own(tiles, 1) : grid_for(tiles);
  if (U == 4) launch_tf1_vec_u<FROM64, OUT, 4>(n, grid, st, out, f, nvec, cp, compress);
  else if (U == 2) launch_tf1_vec_u<FROM64, OUT, 2>(n, grid, st, out, f, nvec, cp, compress);
  else launch_tf1_vec_u<FROM64, OUT, 1>(n, grid, st, out, f, nvec, cp, compress);
}

// One TF1 pass of 1..CFA_MAX_FANIN neighbours over [0, P): `head` scalar elements, a float4
// body of nvec vectors, a scalar tail. out_mode: kOutF32 (last pass, fp32 out), kOutScratch64
// (fp64 scratch of a chained pass) or kOutF64 (last pass, unrounded fp64 out).
static int tf1_pass(void* out, int out_mode, const float* local, const double* w64,
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
    return out_mode != kOutF32 ? (void*)((double*)out + b) : (void*)((float*)out + b);
  };
  auto shifted = [&](size_t b) {
    CompressParams c = cp;
    c.cbegin = cp.cbegin - (long long)b;
    c.cend = cp.cend - (long long)b;
    return c;
  };
  if (nvec > 0) {
    const Tf1Fanin f = fanin_at(head);
    // the fp64-output (wide) form runs one workgroup per CU: 0.749 against 0.729 of peak on the
    // same buffers (tools/kernel_rooflines.py --bpc-variants 2,1); the fp32 outputs keep two
    const CompressParams c = shifted(head);
    void* o = out_at(head);
    const long long nv = (long long)nvec;
    if (out_mode == kOutF32) {
      if (w64) launch_tf1_vec<true, kOutF32>(m, st, o, f, nv, c, compress);
      else launch_tf1_vec<false, kOutF32>(m, st, o, f, nv, c, compress);
    } else if (out_mode == kOutScratch64) {
      if (w64) launch_tf1_vec<true, kOutScratch64>(m, st, o, f, nv, c, compress);
      else launch_tf1_vec<false, kOutScratch64>(m, st, o, f, nv, c, compress);
    } else {
      if (w64) launch_tf1_vec<true, kOutF64>(m, st, o, f, nv, c, compress);
      else launch_tf1_vec<false, kOutF64>(m, st, o, f, nv, c, compress);
    }
    if (int rc = check_launch("mix_tf1_vec")) return rc;
  }
  const size_t tail_begin = head + nvec * 4;
  const size_t pieces[2][2] = {{0, head}, {tail_begin, P}};
  for (auto& pc : pieces) {
    const size_t b = pc[0], e = pc[1];
    if (e <= b) continue;
    const long long len = (long long)(e - b);
    mix_tf1_scalar_kernel<<<grid_for((len + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        out_at(b), out_mode, fanin_at(b), m, len, shifted(b), compress);
    if (int rc = check_launch("mix_tf1_scalar")) return rc;
  }
  return CFA_OK;
}

}  // namespace

extern "C" int cfa_mix_tf1_f32(float* out, const float* local, const float* const* nbrs,
                               const double* alphas, int n, size_t P, int mode, size_t cbegin,
                               size_t cend, unsigned long long* kept_count, void* stream) {
  return cfa_mix_tf1_ex_f32(out, local, nbrs, alphas, n, P, mode, cbegin, cend, kept_count, nullptr,
                            stream);
}

namespace {
// The TF1 chain over fp32 buckets: out is fp32 (rounded once, out64 false) or fp64 (unrounded).
int mix_tf1_impl(void* out, bool out64, const float* local, const float* const* nbrs, const double* alphas,
                 int n, size_t P, int mode, size_t cbegin, size_t cend, unsigned long long* kept_count,
                 double* scratch_in, hipStream_t st, const char* fn) {
  if (n > 0 && !alphas) return fail(CFA_E_INVALID, "%s: null alphas", fn);
  if (mode != CFA_COMPRESS_NONE && !kept_count) return fail(CFA_E_INVALID, "%s: null kept_count", fn);
  // With a counter the epilogue runs (mode 0 keeps, and counts, every element of the range).
  if (cbegin > cend || cend > P) return fail(CFA_E_INVALID, "%s: bad compression range", fn);
  if (out64 && n == 0) return fail(CFA_E_INVALID, "%s: needs at least one neighbour", fn);
  // null pointers, and an output that starts at a neighbour bucket (fp32 or fp64 alike)
  if (int rc = validate_mix(static_cast<const float*>(out), local, nbrs, n, P)) return rc;
  if (out64 && P > 0) {
    // an fp64 out is 8P bytes: each lane's store would overwrite fp32 inputs other lanes have not
    // read yet, so it must not overlap any input range at all (local included)
    const uintptr_t o0 = addr(out), o1 = o0 + P * sizeof(double);
    auto overlaps = [&](const float* x) { return addr(x) < o1 && o0 < addr(x) + P * sizeof(float); };
    if (overlaps(local)) return fail(CFA_E_INVALID, "%s: fp64 out overlaps local", fn);
    for (int j = 0; j < n; ++j)
      if (overlaps(nbrs[j])) return fail(CFA_E_INVALID, "%s: fp64 out overlaps neighbour %d", fn, j);
  }
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  cp.cbegin = (long long)cbegin;
  cp.cend = (long long)cend;
  cp.kept = kept_count;
  const int compress = kept_count ? 1 : 0;
  if (n == 0) {
    // No neighbour: the bucket is the local model (fp32), then the epilogue (cfa_ongraphs.py:218-223).
    float* o = static_cast<float*>(out);
    if (o != local && P > 0)
      CFA_HIP_CHECK(hipMemcpyAsync(o, local, P * sizeof(float), hipMemcpyDefault, st));
    if (!compress) return CFA_OK;
    return cfa_compress_epilogue_f32(o + cbegin, local + cbegin, mode, cend - cbegin, kept_count, st);
  }
  if (P == 0) return CFA_OK;
  // Body/head/tail split shared by every pass (the fp32 pointers decide it; fp64 buckets, the
  // scratch and an fp64 out, are indexed like the bucket and only need 8-byte alignment).
  const uintptr_t mis = addr(out64 ? (const void*)local : out) & 15;
  bool same = (addr(local) & 15) == mis;
  for (int j = 0; j < n; ++j) same = same && ((addr(nbrs[j]) & 15) == mis);
  size_t head = P, nvec = 0;
  if (same && (mis & 3) == 0) {
    head = mis ? (16 - mis) / 4 : 0;
    if (head > P) head = P;
    nvec = (P - head) / 4;
  }
  // chained passes carry w in fp64: in an fp64 out itself, else in the scratch bucket
  double* scratch = out64 ? static_cast<double*>(out) : scratch_in;
  bool owned = false;
  if (n > CFA_MAX_FANIN && !scratch) {
    // no caller scratch: a stream-ordered allocation, which a hipGraph capture must not contain
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    CFA_HIP_CHECK(hipStreamIsCapturing(st, &cs));
    if (cs != hipStreamCaptureStatusNone)
      return fail(CFA_E_INVALID, "%s: %d > %d neighbours under graph capture need a caller scratch "
                  "bucket (cfa_mix_tf1_ex_f32)", fn, n, CFA_MAX_FANIN);
    CFA_HIP_CHECK(hipMallocAsync((void**)&scratch, P * sizeof(double), st));
    owned = true;
  }
  // The vector kernel stores an fp64 output (the fp64 out, or the scratch of chained passes) as
  // 16-B vectors, so that output's body must start 16-B aligned; such buckets only promise 8 B
  // (an fp64 view at an odd element), and then the scalar kernel takes the whole bucket.
  auto body16 = [&](const void* p) { return ((addr(p) + 8 * head) & 15) == 0; };
  if (nvec && ((out64 && !body16(out)) || (n > CFA_MAX_FANIN && !body16(scratch)))) {
    head = P;
    nvec = 0;
  }
  int rc = CFA_OK;
  for (int done = 0; done < n && rc == CFA_OK;) {
    const int m = (n - done) > CFA_MAX_FANIN ? CFA_MAX_FANIN : (n - done);
    const bool last = done + m == n;
    const int out_mode = !last ? kOutScratch64 : (out64 ? kOutF64 : kOutF32);
    rc = tf1_pass(last ? out : (void*)scratch, out_mode, local, done ? scratch : nullptr, nbrs + done,
                  alphas + done, m, P, head, nvec, cp, last ? compress : 0, st);
    done += m;
  }
  if (owned) {
    hipError_t e = hipFreeAsync(scratch, st);
    if (rc == CFA_OK && e != hipSuccess) return fail(CFA_E_HIP, "hipFreeAsync: %s", hipGetErrorString(e));
  }
  return rc;
}
}  // namespace

extern "C" int cfa_mix_tf1_ex_f32(float* out, const float* local, const float* const* nbrs,
                                  const double* alphas, int n, size_t P, int mode, size_t cbegin,
                                  size_t cend, unsigned long long* kept_count, double* scratch_in,
                                  void* stream) {
  return mix_tf1_impl(out, false, local, nbrs, alphas, n, P, mode, cbegin, cend, kept_count, scratch_in,
                      (hipStream_t)stream, "cfa_mix_tf1_f32");
}

extern "C" int cfa_mix_tf1_wide_f32(double* out, const float* local, const float* const* nbrs,
                                    const double* alphas, int n, size_t P, int mode, size_t cbegin,
                                    size_t cend, unsigned long long* kept_count, void* stream) {
  return mix_tf1_impl(out, true, local, nbrs, alphas, n, P, mode, cbegin, cend, kept_count, nullptr,
                      (hipStream_t)stream, "cfa_mix_tf1_wide_f32");
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
      f.r[j + 1] = 1.0 / f.d[j + 1];
    }
    f.fast_div = 1;
    for (int j = 1; j <= m; ++j)
      if (!(f.d[j] >= 0x1p-20 && f.d[j] <= 0x1p20)) f.fast_div = 0;
    const int s0 = done == 0 ? step0_f32 : 0;
    const int cmp = last ? compress : 0;
    bool aligned = m >= 1 && (addr(out) & 15) == 0 && (addr(w) & 15) == 0 && (!cmp || (addr(local) & 15) == 0);
    for (int j = 1; j <= m; ++j) aligned = aligned && (addr(f.src[j]) & 15) == 0;
    long long nvec2 = aligned ? (long long)P / 2 : 0;
    if (nvec2 > 0) {  // 16-byte body on the vector kernel, the odd last element on the scalar one
      const long long tiles = (nvec2 + 2LL * kBlock - 1) / (2LL * kBlock);
      const unsigned vgrid = grid_for(tiles);
      if (rule == CFA_RULE_SEQUENTIAL && s0)
        launch_fold_vec<CFA_RULE_SEQUENTIAL, true>(m, vgrid, st, out, f, nvec2, local, cp, cmp);
      else if (rule == CFA_RULE_SEQUENTIAL)
        launch_fold_vec<CFA_RULE_SEQUENTIAL, false>(m, vgrid, st, out, f, nvec2, local, cp, cmp);
      else if (rule == CFA_RULE_SEQUENTIAL_DIV)
        launch_fold_vec<CFA_RULE_SEQUENTIAL_DIV, false>(m, vgrid, st, out, f, nvec2, local, cp, cmp);
      else
        launch_fold_vec<CFA_RULE_ACCUMULATE, false>(m, vgrid, st, out, f, nvec2, local, cp, cmp);
      if (int rc = check_launch("fold_f64_vec")) return rc;
    }
    const long long b = 2 * nvec2;
    if (b < (long long)P) {
      F64Fanin ft = f;
      for (int j = 0; j <= m; ++j) ft.src[j] = f.src[j] + b;
      CompressParams ct = cp;
      ct.cbegin = cp.cbegin - b;
      ct.cend = cp.cend - b;
      mix_tf1_f64_kernel<<<b ? 1u : grid, kBlock, 0, st>>>(out + b, ft, (long long)P - b, rule, s0, local + b, ct,
                                                          cmp);
      if (int rc = check_launch("fold_f64")) return rc;
    }
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
    bool vec = (addr(W) & 15) == 0;
    for (int j = 0; j < m; ++j)
      vec = vec && a.gstride[j] == 1 && (addr(a.s[j]) & 15) == 0 && (addr(a.g[j]) & 15) == 0;
    const long long nvec2 = vec ? (long long)P / 2 : 0;
    if (nvec2 > 0) {
      // one workgroup per CU: 0.733 against 0.714 of peak on the same buffers (--bpc-variants 2,1)
      launch_mewma_f64_vec(m, grid_for_own((nvec2 + kBlock - 1) / kBlock, 1), st, a, nvec2,
                           std::make_integer_sequence<int, CFA_MAX_FANIN>{});
      if (int rc = check_launch("mewma_tf1_f64_vec")) return rc;
    }
    if (2 * nvec2 < (long long)P) {  // unaligned / strided buckets, or the odd last element
      MewmaF64Args t = a;
      const long long b = 2 * nvec2;
      t.W = a.W + b;
      for (int j = 0; j < m; ++j) {
        t.s[j] = a.s[j] + b;
        t.g[j] = a.g[j] + b * a.gstride[j];
      }
      t.split = a.split - b;
      mewma_tf1_f64_kernel<<<grid_for(((long long)P - b + kBlock - 1) / kBlock), kBlock, 0, st>>>(
          t, (long long)P - b);
      if (int rc = check_launch("mewma_tf1_f64")) return rc;
    }
    done += m;
  }
  return CFA_OK;
}

