// cfa_grad.hip — CFA-GE neighbour-gradient evaluation: the gradient of a device's
// own cost at each neighbour's model, for the two TF1 graphs of cfa_ge_2stage.py, batched over
// the neighbour models in one launch (one workgroup per model).
//
// The reference builds the graph once per call (TF1/consensus/cfa_ge_2stage.py:391-433) and runs
// one Session per neighbour model (:512-528); cfa_ge_4stage.py:391-433 is the same graph.
//   CNN (ML_model 1, :392-405): x[B,L] -> conv1d(W1[F,1,NC], stride S, SAME) + b1 -> relu ->
//       max_pooling1d(pool S, stride S, SAME) -> flatten NWC [B, L2*NC] -> softmax(. W2 + b2)
//   2NN (ML_model 2, :407-420): softmax(relu(x W1 + b1) W2 + b2)
//   cost = mean_b(-sum_c y * log(clip(pred, 1e-15, 0.99))) (:425-426); d cost / d{W1,b1,W2,b2} (:429-430)
// TF conventions kept: SAME padding (out = ceil(L/S), total pad max((out-1)S + k - L, 0), left =
// total/2, padded pooling entries never win), max-pool gradient to the first maximum of a window,
// relu gradient where the activation is > 0, clip gradient where 1e-15 <= pred <= 0.99.
//
// These are tiny latency-bound graphs (P = 1 488 and 16 680 parameters, 24 samples per device):
// each workgroup keeps its model and every activation in LDS and runs forward and backward with
// barriers between the phases. fp32 throughout, like the reference's placeholders.
#include <algorithm>

#include "cfa_internal.h"

namespace {

constexpr float kClipLo = 1e-15f, kClipHi = 0.99f;

// Phase timestamps for tools/probe/grad_phases.hip (compiled out of the library).
#ifdef CFA_GRAD_PHASES
// Stamps go to LDS and are copied out at the last phase (8 / 17), so no phase waits on the
// previous stamp's global store.
__device__ unsigned long long g_phase[32];
__device__ unsigned long long g_wg[4096][2];  // per workgroup: first and last stamp
__device__ __forceinline__ unsigned long long* phase_lds() {
  __shared__ unsigned long long s[32];  // one array per kernel, shared by every PHASE site
  return s;
}
#define PHASE(k) \
  do {           \
    unsigned long long* s_ts_ = phase_lds(); \
    __syncthreads(); \
    if (threadIdx.x == 0) { \
      s_ts_[k] = wall_clock64(); \
      if ((k) == 8 || (k) == 17) { \
        const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x; \
        const int k0_ = (k) == 8 ? 0 : 10; \
        if (blockIdx.x == 0 && blockIdx.y == 0) \
          for (int j_ = k0_; j_ <= (k); ++j_) g_phase[j_] = s_ts_[j_]; \
        if (wg_ < 4096) g_wg[wg_][0] = s_ts_[k0_], g_wg[wg_][1] = s_ts_[k]; \
      } \
    } \
  } while (0)
#else
#define PHASE(k) \
  do {           \
  } while (0)
#endif

__host__ __device__ inline int same_left(int L, int k, int s) {
  const int out = (L + s - 1) / s;
  const int total = max((out - 1) * s + k - L, 0);
  return total / 2;
}

// Softmax + clipped cross-entropy backward, in place on logits z[nb][C] -> d logits:
// d cost / d pred_c = -(y_c / clip(pred_c)) / B where the clip passes the gradient; then the
// softmax gradient (dp - sum(dp * p)) * p (TF SoftmaxGrad). One lane per class: a sample's
// W >= C lanes (W a power of two <= 64, so a group never straddles a wave) reduce max, sum and
// dot with xor shuffles, and every value stays in registers.
__device__ void softmax_xent_backward(float* z, const float* y, int nb, int C, int W, float invB, int tid,
                                      int T) {
  for (int idx = tid; idx < nb * W; idx += T) {
    const int b = idx / W, c = idx % W;
    const bool valid = c < C;
    const float zc = valid ? z[b * C + c] : -INFINITY;
    const float yc = valid ? y[b * C + c] : 0.f;
    float mx = zc;
    for (int o = W >> 1; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, W));
    const float e = valid ? expf(zc - mx) : 0.f;
    float s = e;
    for (int o = W >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, W);
    const float p = e / s;  // pred
    const bool pass = valid && p >= kClipLo && p <= kClipHi;
    const float dp = pass ? -(yc / fminf(fmaxf(p, kClipLo), kClipHi)) * invB : 0.f;
    float dot = dp * p;
    for (int o = W >> 1; o > 0; o >>= 1) dot += __shfl_xor(dot, o, W);
    if (valid) z[b * C + c] = (dp - dot) * p;
  }
}

// lanes per sample of softmax_xent_backward: the power of two >= C (C <= 64, checked on the host)
inline int softmax_width(int C) {
  int w = 1;
  while (w < C) w <<= 1;
  return w;
}

constexpr int kGradBlock = 512;  // 8 waves: these graphs are latency-bound, not ALU-bound

// Copy n floats global -> LDS with every load of a thread issued before its first store (the
// graphs are tiny, so serialized global latency, not bandwidth, would dominate). The tail is
// predicated rather than looped, so a copy of up to U * T floats is one round trip.
__device__ __forceinline__ void stage(float* dst, const float* src, int n, int tid, int T) {
  constexpr int U = 8;
  for (int i = tid; i < n; i += U * T) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * T < n ? src[i + u * T] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * T < n) dst[i + u * T] = v[u];
  }
}

// stage() of three segments with all their loads in flight together.
__device__ __forceinline__ void stage3(float* d0, const float* s0, int n0, float* d1, const float* s1, int n1,
                                       float* d2, const float* s2, int n2, int tid, int T) {
  constexpr int U = 4;
  const int n = max(n0, max(n1, n2));
  for (int i = tid; i < n; i += U * T) {
    float v0[U], v1[U], v2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + u * T;
      v0[u] = j < n0 ? s0[j] : 0.f;
      v1[u] = j < n1 ? s1[j] : 0.f;
      v2[u] = j < n2 ? s2[j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + u * T;
      if (j < n0) d0[j] = v0[u];
      if (j < n1) d1[j] = v1[u];
      if (j < n2) d2[j] = v2[u];
    }
  }
}

constexpr int kMaxTaps = 32;  // conv filter taps held in registers (larger filters read LDS)

struct CnnDims {
  int B, L, C, F, NC, S;
  int SW;              // softmax lanes per sample (softmax_width(C))
  int L1, L2, pl, ql;  // conv / pool output lengths, left pads
  int Bc;              // samples per LDS-resident chunk
  int Bs;              // samples per workgroup (grid.y splits the batch; partial sums go to a workspace)
  long long P;         // parameters per model
};

// Per-sample LDS floats of the CNN kernel: x row, pooled / argmax / d pooled, logits, and the
// per-sample partial sums of the conv-layer gradients.
inline long long cnn_lds_per_sample(const CnnDims& d) {
  const long long LN = (long long)d.L2 * d.NC;
  return d.L + 3 * LN + 2LL * d.C + (long long)d.F * d.NC + d.NC;
}
inline long long cnn_lds_fixed(const CnnDims& d) {
  const long long LN = (long long)d.L2 * d.NC;
  return (long long)d.F * d.NC + d.NC + LN * d.C + d.C;
}

// Gradient sums run over all B samples; samples go through LDS in chunks of Bc. Every output
// element is owned by one thread for the whole launch (the same index loop in every chunk), so
// the per-chunk sums accumulate in the output bucket without atomics, in a fixed order.
// FT, ST > 0: a filter of FT taps with stride (= pool size) ST at compile time: an interior
// pooling window's (ST - 1) * ST + FT input samples are loaded once, all in flight together, and
// its ST convolutions run from registers. FT = ST = 0: any geometry (runtime loops).
template <int FT, int ST>
__global__ __launch_bounds__(kGradBlock) void grad_cnn_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ y,
                                                              const float* __restrict__ models,
                                                              const int* __restrict__ mrow,
                                                              const int* __restrict__ drow,
                                                              float* __restrict__ grads, CnnDims d) {
  extern __shared__ float lds[];
  const int LN = d.L2 * d.NC;
  const int nW1 = d.F * d.NC, nW2 = LN * d.C, nG1 = nW1 + d.NC;
  float* W1 = lds;                        // [F][NC]
  float* b1 = W1 + nW1;                   // [NC]
  float* W2 = b1 + d.NC;                  // [LN][C]
  float* b2 = W2 + nW2;                   // [C]
  float* xs = b2 + d.C;                   // [Bc][L]
  float* pooled = xs + d.Bc * d.L;        // [Bc][L2][NC]
  int* arg = reinterpret_cast<int*>(pooled + d.Bc * LN);  // conv position of each window's max
  float* dfc = reinterpret_cast<float*>(arg + d.Bc * LN); // [Bc][LN]
  float* zl = dfc + d.Bc * LN;            // [Bc][C]: logits, then d logits
  float* ys = zl + d.Bc * d.C;            // [Bc][C] labels
  float* part = ys + d.Bc * d.C;          // [Bc][nG1]: per-sample conv-gradient sums
  // model and data rows of this workgroup's evaluation (population form), else model blockIdx.x
  // on the one data set
  const float* m = models + (long long)(mrow ? mrow[blockIdx.x] : (int)blockIdx.x) * d.P;
  const long long dr = drow ? drow[blockIdx.x] : 0;
  x += dr * d.B * d.L;
  y += dr * d.B * d.C;
  // grid.y splits the batch: this workgroup sums samples [bb, be) into its own partial bucket
  // (gridDim.y == 1: the model's gradient bucket itself)
  float* g = grads + ((long long)blockIdx.x * gridDim.y + blockIdx.y) * d.P;
  const int bb = blockIdx.y * d.Bs, be = min(d.B, bb + d.Bs);
  const int tid = threadIdx.x, T = blockDim.x;
  float* gW2 = g + nG1;
  float* gb2 = gW2 + nW2;
  const float invB = 1.0f / (float)d.B;

  PHASE(0);
  // the model bucket (W1 b1 W2 b2) and the first chunk's samples and labels, all in flight
  // together: one global round trip before the first barrier
  stage3(W1, m, nG1 + nW2 + d.C, xs, x + (long long)bb * d.L, bb < be ? min(d.Bc, be - bb) * d.L : 0, ys,
         y + (long long)bb * d.C, bb < be ? min(d.Bc, be - bb) * d.C : 0, tid, T);
  __syncthreads();
  PHASE(1);
  // the conv taps of this thread's channel stay in registers (T is a multiple of NC, so every
  // item a thread takes below has the same channel c = tid % NC)
  const bool taps_in_regs = d.F <= kMaxTaps && T % d.NC == 0;
  float wreg[kMaxTaps];
  {
    // one channel index and one uniform branch around every tap load (a per-tap predicate
    // recomputed the modulo and branched 32 times: 2.6 us at the config-3 shapes)
    const int creg = tid % d.NC;
    constexpr int KT = FT > 0 ? FT : kMaxTaps;
#pragma unroll
    for (int k = 0; k < kMaxTaps; ++k) wreg[k] = 0.f;
    if (taps_in_regs) {
#pragma unroll
      for (int k = 0; k < KT; ++k)
        if (FT > 0 || k < d.F) wreg[k] = W1[k * d.NC + creg];
    }
  }
  if (bb >= be) {  // no sample left for this split: a zero partial
    for (long long i = threadIdx.x; i < d.P; i += blockDim.x) g[i] = 0.f;
    return;
  }
  for (int b0 = bb; b0 < be; b0 += d.Bc) {
    const int nb = min(d.Bc, be - b0);
    const bool first = b0 == bb;
    if (!first) {  // the first chunk was staged with the model
      stage(xs, x + (long long)b0 * d.L, nb * d.L, tid, T);
      stage(ys, y + (long long)b0 * d.C, nb * d.C, tid, T);
      __syncthreads();
    }
    PHASE(2);
    // conv + bias + relu evaluated inside each pooling window; keep the max and its position
    for (int idx = tid; idx < nb * LN; idx += T) {
      const int b = idx / LN, r = idx % LN, q = r / d.NC, c = r % d.NC;
      const float* xb = xs + b * d.L;
      float best = -INFINITY;
      int barg = -1;
      bool done = false;
      if constexpr (FT > 0 && ST > 0) {
        // Every window, boundary ones included, takes this branch-free path: samples outside
        // [0, L) read as 0 (a zero tap adds nothing: fma(0, w, z) == z) and positions outside
        // [0, L1) never win, so no lane of a wave waits on a divergent slow path.
        constexpr int NX = (ST - 1) * ST + FT;
        const int p0 = q * ST - d.ql, t0 = p0 * ST - d.pl;
        if (taps_in_regs) {
          float xv[NX];
#pragma unroll
          for (int u = 0; u < NX; ++u) {
            const int t = t0 + u;
            const bool in = t >= 0 && t < d.L;
            const float v = xb[in ? t : 0];
            xv[u] = in ? v : 0.f;
          }
#pragma unroll
          for (int j = 0; j < ST; ++j) {
            float z = 0.f;
#pragma unroll
            for (int k = 0; k < FT; ++k) z = fmaf(xv[j * ST + k], wreg[k], z);
            z += b1[c];
            const float h = z > 0.f ? z : 0.f;
            const int p = p0 + j;
            if (p >= 0 && p < d.L1 && h > best) {
              best = h;
              barg = p;
            }
          }
          done = true;
        }
      }
      for (int j = 0; j < d.S && !done; ++j) {
        const int p = q * d.S - d.ql + j;
        if (p < 0 || p >= d.L1) continue;
        const int t0 = p * d.S - d.pl;
        float z = 0.f;
        for (int k = 0; k < d.F; ++k) {
          const int t = t0 + k;
          if (t >= 0 && t < d.L) z = fmaf(xb[t], W1[k * d.NC + c], z);
        }
        z += b1[c];
        const float h = z > 0.f ? z : 0.f;
        if (h > best) {
          best = h;
          barg = p;
        }
      }
      pooled[idx] = best;
      arg[idx] = barg;
    }
    __syncthreads();
    PHASE(3);
    // logits: 8 lanes per (sample, class), strided partial sums, xor-shuffle reduction
    for (int idx = tid; idx < nb * d.C * 8; idx += T) {
      const int o = idx >> 3, lane = idx & 7;
      const int b = o / d.C, k = o % d.C;
      float z = 0.f;
      for (int i = lane; i < LN; i += 8) z = fmaf(pooled[b * LN + i], W2[i * d.C + k], z);
      z += __shfl_xor(z, 1, 8);
      z += __shfl_xor(z, 2, 8);
      z += __shfl_xor(z, 4, 8);
      if (lane == 0) zl[o] = z + b2[k];
    }
    __syncthreads();
    PHASE(4);
    softmax_xent_backward(zl, ys, nb, d.C, d.SW, invB, tid, T);
    __syncthreads();
    PHASE(5);

    // dense layer gradients and the gradient flowing into the pooled features
    for (int idx = tid; idx < nW2; idx += T) {
      const int i = idx / d.C, k = idx % d.C;
      float s = first ? 0.f : gW2[idx];
#pragma unroll 8
      for (int b = 0; b < nb; ++b) s = fmaf(pooled[b * LN + i], zl[b * d.C + k], s);
      gW2[idx] = s;
    }
    for (int k = tid; k < d.C; k += T) {
      float s = first ? 0.f : gb2[k];
      for (int b = 0; b < nb; ++b) s += zl[b * d.C + k];
      gb2[k] = s;
    }
    for (int idx = tid; idx < nb * LN; idx += T) {
      const int b = idx / LN, i = idx % LN;
      float s = 0.f;
      for (int k = 0; k < d.C; ++k) s = fmaf(zl[b * d.C + k], W2[i * d.C + k], s);
      dfc[idx] = pooled[idx] > 0.f ? s : 0.f;  // relu gradient at the window's max
    }
    __syncthreads();
    PHASE(6);
    // conv gradients per (weight, sample): only each window's max position receives gradient
    for (int idx = tid; idx < nG1 * nb; idx += T) {  // e fastest: lanes read neighbouring channels
      const int e = idx % nG1, b = idx / nG1;
      float s = 0.f;
      if (e < nW1) {
        const int k = e / d.NC, c = e % d.NC;
#pragma unroll 7
        for (int q = 0; q < d.L2; ++q) {  // select, not branch: the loads stay in flight together
          const int f = b * LN + q * d.NC + c;
          const int t = arg[f] * d.S + k - d.pl;
          const bool in = t >= 0 && t < d.L;
          const float xv = xs[b * d.L + (in ? t : 0)];
          s = fmaf(dfc[f], in ? xv : 0.f, s);
        }
      } else {
        const int c = e - nW1;
#pragma unroll 7
        for (int q = 0; q < d.L2; ++q) s += dfc[b * LN + q * d.NC + c];
      }
      part[b * nG1 + e] = s;
    }
    __syncthreads();
    PHASE(7);
    for (int e = tid; e < nG1; e += T) {  // sum over the chunk's samples in order
      float s = first ? 0.f : g[e];
      for (int b = 0; b < nb; ++b) s += part[b * nG1 + e];
      g[e] = s;
    }
    __syncthreads();  // the chunk's LDS is reused by the next one
    PHASE(8);
  }
}

constexpr int kSpan = 32;  // first-layer inputs per partial sum (W1 slice held in registers)

struct NnDims {
  int B, L, H, C;
  int SW;  // softmax lanes per sample (softmax_width(C))
  int G;   // ceil(L / kSpan) slices of the input dimension for the first layer's partial sums
  int Bc;
  int Bs;  // samples per workgroup (grid.y splits the batch; partial sums go to a workspace)
  long long P;
};

inline long long nn_lds_per_sample(const NnDims& d) { return d.L + 2LL * d.H + 2LL * d.C + (long long)d.G * d.H; }
inline long long nn_lds_fixed(const NnDims& d) { return d.H + (long long)d.H * d.C + d.C; }

__global__ __launch_bounds__(kGradBlock) void grad_2nn_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ y,
                                                              const float* __restrict__ models,
                                                              const int* __restrict__ mrow,
                                                              const int* __restrict__ drow,
                                                              float* __restrict__ grads, NnDims d) {
  extern __shared__ float lds[];
  float* b1 = lds;                 // [H]
  float* W2 = b1 + d.H;            // [H][C]
  float* b2 = W2 + d.H * d.C;      // [C]
  float* xs = b2 + d.C;            // [Bc][L]
  float* act = xs + d.Bc * d.L;    // [Bc][H] relu(x W1 + b1)
  float* dz = act + d.Bc * d.H;    // [Bc][H]
  float* zl = dz + d.Bc * d.H;     // [Bc][C]
  float* ys = zl + d.Bc * d.C;     // [Bc][C]
  float* zpart = ys + d.Bc * d.C;  // [G][Bc][H]
  const long long nW1 = (long long)d.L * d.H;
  const float* m = models + (long long)(mrow ? mrow[blockIdx.x] : (int)blockIdx.x) * d.P;
  const long long dr = drow ? drow[blockIdx.x] : 0;
  x += dr * d.B * d.L;
  y += dr * d.B * d.C;
  const float* W1 = m;             // [L][H], read from global once per launch (kept in registers)
  // grid.y splits the batch: this workgroup sums samples [bb, be) into its own partial bucket
  // (gridDim.y == 1: the model's gradient bucket itself)
  float* g = grads + ((long long)blockIdx.x * gridDim.y + blockIdx.y) * d.P;
  const int bb = blockIdx.y * d.Bs, be = min(d.B, bb + d.Bs);
  float* gW1 = g;
  float* gb1 = gW1 + nW1;
  float* gW2 = gb1 + d.H;
  float* gb2 = gW2 + d.H * d.C;
  const int tid = threadIdx.x, T = blockDim.x;
  const float invB = 1.0f / (float)d.B;
  const int H4 = (d.H % 4 == 0 && (reinterpret_cast<uintptr_t>(dz) & 15) == 0) ? d.H / 4 : 0;

  PHASE(10);
  // W1 slice of this thread's (slice, h) pairs: with G * H <= T every thread owns one pair and
  // loads its kSpan weights once. These loads, the rest of the model (b1 W2 b2) and the first
  // chunk's samples and labels are all in flight together: one global round trip.
  const bool w_in_regs = d.G * d.H <= T;
  float wreg[kSpan];
  {
    const int h = tid % d.H, grp = tid / d.H, i0 = grp * kSpan;
#pragma unroll
    for (int u = 0; u < kSpan; ++u)
      wreg[u] = (w_in_regs && grp < d.G && i0 + u < d.L) ? W1[(long long)(i0 + u) * d.H + h] : 0.f;
  }
  stage3(b1, m + nW1, d.H + d.H * d.C + d.C, xs, x + (long long)bb * d.L, bb < be ? min(d.Bc, be - bb) * d.L : 0,
         ys, y + (long long)bb * d.C, bb < be ? min(d.Bc, be - bb) * d.C : 0, tid, T);
  if (bb >= be) {  // no sample left for this split: a zero partial
    for (long long i = threadIdx.x; i < d.P; i += blockDim.x) g[i] = 0.f;
    return;
  }
  for (int b0 = bb; b0 < be; b0 += d.Bc) {
    const int nb = min(d.Bc, be - b0);
    const bool first = b0 == bb;
    if (!first) {  // the first chunk was staged with the model
      stage(xs, x + (long long)b0 * d.L, nb * d.L, tid, T);
      stage(ys, y + (long long)b0 * d.C, nb * d.C, tid, T);
    }
    __syncthreads();
    PHASE(11);
    // first layer as G partial sums over kSpan-wide slices of the input dimension
    if (w_in_regs) {
      const int h = tid % d.H, grp = tid / d.H, i0 = grp * kSpan;
      if (grp < d.G) {
        for (int b = 0; b < nb; ++b) {
          const float* xb = xs + b * d.L + i0;
          float z = 0.f;
          if (i0 + kSpan <= d.L) {  // full slice: every load issued before the FMA chain
            float xv[kSpan];
#pragma unroll
            for (int u = 0; u < kSpan; ++u) xv[u] = xb[u];
#pragma unroll
            for (int u = 0; u < kSpan; ++u) z = fmaf(xv[u], wreg[u], z);
          } else {
#pragma unroll
            for (int u = 0; u < kSpan; ++u)
              if (u < d.L - i0) z = fmaf(xb[u], wreg[u], z);
          }
          zpart[(grp * d.Bc + b) * d.H + h] = z;
        }
      }
    } else {
      for (int idx = tid; idx < d.G * nb * d.H; idx += T) {
        const int h = idx % d.H, r = idx / d.H, b = r % nb, grp = r / nb;
        const int i0 = grp * kSpan, i1 = min(d.L, i0 + kSpan);
        float z = 0.f;
        for (int i = i0; i < i1; ++i) z = fmaf(xs[b * d.L + i], W1[(long long)i * d.H + h], z);
        zpart[(grp * d.Bc + b) * d.H + h] = z;
      }
    }
    __syncthreads();
    PHASE(12);
    for (int idx = tid; idx < nb * d.H; idx += T) {
      const int b = idx / d.H, h = idx % d.H;
      float z = 0.f;
      for (int grp = 0; grp < d.G; ++grp) z += zpart[(grp * d.Bc + b) * d.H + h];
      z += b1[h];
      act[idx] = z > 0.f ? z : 0.f;
    }
    __syncthreads();
    PHASE(13);
    for (int idx = tid; idx < nb * d.C; idx += T) {
      const int b = idx / d.C, k = idx % d.C;
      float z = 0.f;
      for (int h = 0; h < d.H; ++h) z = fmaf(act[b * d.H + h], W2[h * d.C + k], z);
      zl[idx] = z + b2[k];
    }
    __syncthreads();
    PHASE(14);
    softmax_xent_backward(zl, ys, nb, d.C, d.SW, invB, tid, T);
    __syncthreads();
    PHASE(15);
    for (int idx = tid; idx < d.H * d.C; idx += T) {
      const int h = idx / d.C, k = idx % d.C;
      float s = first ? 0.f : gW2[idx];
      for (int b = 0; b < nb; ++b) s = fmaf(act[b * d.H + h], zl[b * d.C + k], s);
      gW2[idx] = s;
    }
    for (int k = tid; k < d.C; k += T) {
      float s = first ? 0.f : gb2[k];
      for (int b = 0; b < nb; ++b) s += zl[b * d.C + k];
      gb2[k] = s;
    }
    for (int idx = tid; idx < nb * d.H; idx += T) {
      const int b = idx / d.H, h = idx % d.H;
      float s = 0.f;
      for (int k = 0; k < d.C; ++k) s = fmaf(zl[b * d.C + k], W2[h * d.C + k], s);
      dz[idx] = act[idx] > 0.f ? s : 0.f;
    }
    __syncthreads();
    PHASE(16);
    if (H4) {  // gW1 = x^T dz, four h per thread: one x read feeds four FMAs
      const f4* dz4 = reinterpret_cast<const f4*>(dz);
      f4* gW14 = reinterpret_cast<f4*>(gW1);
      const bool aligned = (reinterpret_cast<uintptr_t>(gW1) & 15) == 0;
      for (long long idx = tid; idx < nW1 / 4; idx += T) {
        const int i = (int)(idx / H4), hq = (int)(idx % H4);
        f4 s;
        if (first) {
          s = f4{0.f, 0.f, 0.f, 0.f};
        } else if (aligned) {
          s = gW14[idx];
        } else {
          for (int c = 0; c < 4; ++c) s[c] = gW1[idx * 4 + c];
        }
#pragma unroll 8
        for (int b = 0; b < nb; ++b) {
          const float xv = xs[b * d.L + i];
          const f4 dv = dz4[b * H4 + hq];
          s.x = fmaf(xv, dv.x, s.x);
          s.y = fmaf(xv, dv.y, s.y);
          s.z = fmaf(xv, dv.z, s.z);
          s.w = fmaf(xv, dv.w, s.w);
        }
        if (aligned) gW14[idx] = s;
        else for (int c = 0; c < 4; ++c) gW1[idx * 4 + c] = s[c];
      }
    } else {
      for (long long idx = tid; idx < nW1; idx += T) {
        const int i = (int)(idx / d.H), h = (int)(idx % d.H);
        float s = first ? 0.f : gW1[idx];
        for (int b = 0; b < nb; ++b) s = fmaf(xs[b * d.L + i], dz[b * d.H + h], s);
        gW1[idx] = s;
      }
    }
    for (int h = tid; h < d.H; h += T) {
      float s = first ? 0.f : gb1[h];
      for (int b = 0; b < nb; ++b) s += dz[b * d.H + h];
      gb1[h] = s;
    }
    __syncthreads();
    PHASE(17);
  }
}

// Dynamic LDS for one workgroup: up to 64 KiB by default; above that the kernel's limit is
// raised to the device's (160 KiB on gfx950) when the runtime allows it.
int device_lds_max() {  // per device, cached after the first query
  static int cache[64] = {0};
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 65536;
  if (dev >= 0 && dev < 64) {
    const int c = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (c > 0) return c;
  }
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || v <= 0) v = 65536;
  if (dev >= 0 && dev < 64) __atomic_store_n(&cache[dev], v, __ATOMIC_RELAXED);
  return v;
}

// Raise a kernel's dynamic-LDS limit to `bytes` once per (kernel, device); false if refused.
bool raise_lds_limit(const void* kernel, int bytes) {
  static const void* keys[8] = {nullptr};
  static int granted[8][64] = {{0}};  // per kernel slot and device: the limit granted so far
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = -1;
  int slot = -1;
  for (int i = 0; i < 8 && dev >= 0; ++i) {
    const void* k = __atomic_load_n(&keys[i], __ATOMIC_ACQUIRE);
    if (k == kernel) { slot = i; break; }
    if (!k) {
      const void* expected = nullptr;
      if (__atomic_compare_exchange_n(&keys[i], &expected, kernel, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE) ||
          expected == kernel) {
        slot = i;
        break;
      }
    }
  }
  if (slot >= 0 && __atomic_load_n(&granted[slot][dev], __ATOMIC_RELAXED) >= bytes) return true;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (slot >= 0) __atomic_store_n(&granted[slot][dev], bytes, __ATOMIC_RELAXED);
  return true;
}

// Samples per chunk for `fixed` + Bc * `per_sample` floats of LDS; sets *bytes. 0 if not even one fits.
int plan_chunk(const void* kernel, long long fixed, long long per_sample, int B, long long* bytes) {
  long long limit = device_lds_max();
  if (const char* cap = getenv("CFA_GRAD_LDS_CAP")) limit = std::min<long long>(limit, atoll(cap));  // measurement knob
  auto fit = [&](long long lim) { return (int)std::min<long long>(B, (lim / 4 - fixed) / per_sample); };
  int bc = fit(limit);
  if (4 * (fixed + per_sample * bc) > 65536 && !raise_lds_limit(kernel, (int)limit)) bc = fit(65536);
  *bytes = 4 * (fixed + per_sample * std::max(bc, 0));
  return std::max(bc, 0);
}

}  // namespace

// Current device: cache its LDS size and raise every gradient kernel's dynamic-LDS limit to it
// now, so later launches (e.g. under hipGraph capture) need no attribute call.
int grad_prepare_device() {
  const int lim = device_lds_max();
  if (lim <= 65536) return CFA_OK;
  const void* kernels[] = {(const void*)grad_cnn_kernel<16, 5>, (const void*)grad_cnn_kernel<0, 0>,
                           (const void*)grad_2nn_kernel};
  for (const void* k : kernels) (void)raise_lds_limit(k, lim);  // refused: launches stay within 64 KiB
  return CFA_OK;
}

namespace {

// Sum of the Sp partial buckets of each evaluation, in split order (deterministic).
__global__ __launch_bounds__(kBlock) void reduce_splits_kernel(const float* __restrict__ ws,
                                                               float* __restrict__ grads, int Sp,
                                                               long long P) {
  const long long m = blockIdx.y;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long long)gridDim.x * kBlock) {
    float s = ws[(m * Sp) * P + i];
    for (int sp = 1; sp < Sp; ++sp) s += ws[(m * Sp + sp) * P + i];
    grads[m * P + i] = s;
  }
}

int launch_reduce_splits(const float* ws, float* grads, int M, int Sp, long long P, hipStream_t st) {
  reduce_splits_kernel<<<dim3((unsigned)std::min<long long>((P + kBlock - 1) / kBlock, 64), (unsigned)M), kBlock, 0,
                         st>>>(ws, grads, Sp, P);
  return check_launch("reduce_splits_kernel");
}

// Batch split for M evaluations of B samples of P-parameter models: about two workgroups per CU
// in all, at most 8 per evaluation, and fewer for larger models, whose partial buckets (written
// and re-read by the reduction) and per-workgroup weight staging grow with P. Measured at the
// CFA-GE shapes (tools/probe/grad_split_sweep.sh, 32 evaluations of 24 samples): CNN (P = 1 488)
// 41.5 -> 17.0 us at 8 splits, 2NN (P = 16 680) 28.5 -> 21.3 us at 3, both slower past that.
int batch_split(int M, int B, long long P) {
  if (M <= 0 || B <= 1) return 1;
  int want = (2 * device_cus() + M - 1) / M;
  want = std::min<long long>(want, std::min<long long>(8, std::max<long long>(1, 65536 / std::max<long long>(P, 1))));
  if (const char* e = getenv("CFA_GRAD_SPLIT")) want = std::max(1, atoi(e));  // measurement knob
  int sp = std::max(1, std::min(B, want));
  const int bs = (B + sp - 1) / sp;
  return (B + bs - 1) / bs;
}

// Workspace of a split launch: the M * Sp partial buckets.
size_t split_workspace_elems(int M, int Sp, long long P) { return (size_t)M * Sp * (size_t)P; }

int launch_grad_cnn(const char* fn, const float* x, const float* y, int B, int L, int classes, int filter,
                    int number, int stride, const float* models, const int* mrow, const int* drow,
                    float* grads, float* ws, size_t ws_elems, int M, void* stream) {
  if (M < 0 || B < 1 || L < 1 || classes < 1 || filter < 1 || number < 1 || stride < 1)
    return fail(CFA_E_INVALID, "%s: bad dimensions (B %d L %d C %d F %d NC %d S %d M %d)", fn, B, L, classes,
                filter, number, stride, M);
  if (M == 0) return CFA_OK;
  if (!x || !y || !models || (!grads && !ws)) return fail(CFA_E_INVALID, "%s: null buffer", fn);
  CnnDims d;
  if (classes > 64) return fail(CFA_E_UNSUPPORTED, "%s: more than 64 classes", fn);
  d.B = B, d.L = L, d.C = classes, d.F = filter, d.NC = number, d.S = stride;
  d.SW = softmax_width(classes);
  d.L1 = (L + stride - 1) / stride;
  d.L2 = (d.L1 + stride - 1) / stride;
  d.pl = same_left(L, filter, stride);
  d.ql = same_left(d.L1, stride, stride);
  d.P = (long long)filter * number + number + (long long)d.L2 * number * classes + classes;
  long long bytes = 0;
  // the CFA-GE CNN's geometry (filter 16, stride 5: federated_sample_CNN_CFA-GE.py:36-39) gets
  // the unrolled kernel
  const bool fast = filter == 16 && stride == 5;
  const void* kern = fast ? (const void*)grad_cnn_kernel<16, 5> : (const void*)grad_cnn_kernel<0, 0>;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int Sp = batch_split(M, B, d.P);
  if (!grads) {  // partials only: [M][Sp][P] into the workspace, summed by the caller
    if (ws_elems < split_workspace_elems(M, Sp, d.P))
      return fail(CFA_E_INVALID, "%s: partials-only launch needs %zu workspace floats", fn,
                  split_workspace_elems(M, Sp, d.P));
  } else if (!ws || ws_elems < split_workspace_elems(M, Sp, d.P)) {
    Sp = 1;
  }
  d.Bs = (B + Sp - 1) / Sp;
  // LDS for the samples one workgroup takes (its split), not the whole batch
  d.Bc = plan_chunk(kern, cnn_lds_fixed(d), cnn_lds_per_sample(d), d.Bs, &bytes);
  if (d.Bc < 1) return fail(CFA_E_UNSUPPORTED, "%s: one sample does not fit the workgroup's LDS", fn);
  float* part = (Sp > 1 || !grads) ? ws : grads;
  const dim3 grid((unsigned)M, (unsigned)Sp);
  if (fast)
    grad_cnn_kernel<16, 5><<<grid, kGradBlock, (size_t)bytes, st>>>(x, y, models, mrow, drow, part, d);
  else
    grad_cnn_kernel<0, 0><<<grid, kGradBlock, (size_t)bytes, st>>>(x, y, models, mrow, drow, part, d);
  if (int rc = check_launch("grad_cnn_kernel")) return rc;
  return (Sp > 1 && grads) ? launch_reduce_splits(ws, grads, M, Sp, d.P, st) : CFA_OK;
}

int launch_grad_2nn(const char* fn, const float* x, const float* y, int B, int L, int hidden, int classes,
                    const float* models, const int* mrow, const int* drow, float* grads, float* ws,
                    size_t ws_elems, int M, void* stream) {
  if (M < 0 || B < 1 || L < 1 || hidden < 1 || classes < 1)
    return fail(CFA_E_INVALID, "%s: bad dimensions (B %d L %d H %d C %d M %d)", fn, B, L, hidden, classes, M);
  if (M == 0) return CFA_OK;
  if (!x || !y || !models || (!grads && !ws)) return fail(CFA_E_INVALID, "%s: null buffer", fn);
  NnDims d;
  if (classes > 64) return fail(CFA_E_UNSUPPORTED, "%s: more than 64 classes", fn);
  d.B = B, d.L = L, d.H = hidden, d.C = classes;
  d.SW = softmax_width(classes);
  d.G = (L + kSpan - 1) / kSpan;
  d.P = (long long)L * hidden + hidden + (long long)hidden * classes + classes;
  long long bytes = 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int Sp = batch_split(M, B, d.P);
  if (!grads) {  // partials only: [M][Sp][P] into the workspace, summed by the caller
    if (ws_elems < split_workspace_elems(M, Sp, d.P))
      return fail(CFA_E_INVALID, "%s: partials-only launch needs %zu workspace floats", fn,
                  split_workspace_elems(M, Sp, d.P));
  } else if (!ws || ws_elems < split_workspace_elems(M, Sp, d.P)) {
    Sp = 1;
  }
  d.Bs = (B + Sp - 1) / Sp;
  // LDS for the samples one workgroup takes (its split), not the whole batch
  d.Bc = plan_chunk((const void*)grad_2nn_kernel, nn_lds_fixed(d), nn_lds_per_sample(d), d.Bs, &bytes);
  if (d.Bc < 1) return fail(CFA_E_UNSUPPORTED, "%s: one sample does not fit the workgroup's LDS", fn);
  float* part = (Sp > 1 || !grads) ? ws : grads;
  grad_2nn_kernel<<<dim3((unsigned)M, (unsigned)Sp), kGradBlock, (size_t)bytes, st>>>(x, y, models, mrow, drow, part,
                                                                                       d);
  if (int rc = check_launch("grad_2nn_kernel")) return rc;
  return (Sp > 1 && grads) ? launch_reduce_splits(ws, grads, M, Sp, d.P, st) : CFA_OK;
}

}  // namespace

extern "C" int cfa_ge_grad_cnn_f32(const float* x, const float* y, int B, int L, int classes,
                                   int filter, int number, int stride, const float* models,
                                   float* grads, int M, void* stream) {
  return launch_grad_cnn("cfa_ge_grad_cnn_f32", x, y, B, L, classes, filter, number, stride, models, nullptr,
                         nullptr, grads, nullptr, 0, M, stream);
}

extern "C" int cfa_ge_grad_2nn_f32(const float* x, const float* y, int B, int L, int hidden,
                                   int classes, const float* models, float* grads, int M,
                                   void* stream) {
  return launch_grad_2nn("cfa_ge_grad_2nn_f32", x, y, B, L, hidden, classes, models, nullptr, nullptr, grads,
                         nullptr, 0, M, stream);
}

extern "C" int cfa_ge_grad_splits(int M, int B, size_t P) { return batch_split(M, B, (long long)P); }

extern "C" size_t cfa_ge_grad_workspace_elems(int M, int B, size_t P) {
  const int sp = batch_split(M, B, (long long)P);
  return sp > 1 ? split_workspace_elems(M, sp, (long long)P) : 0;
}

extern "C" int cfa_ge_grad_cnn_rows_f32(const float* x, const float* y, int B, int L, int classes,
                                        int filter, int number, int stride, const float* models,
                                        const int32_t* model_row, const int32_t* data_row,
                                        float* grads, float* workspace, size_t workspace_elems, int M,
                                        void* stream) {
  if (M > 0 && (!model_row || !data_row))
    return fail(CFA_E_INVALID, "cfa_ge_grad_cnn_rows_f32: null row table");
  return launch_grad_cnn("cfa_ge_grad_cnn_rows_f32", x, y, B, L, classes, filter, number, stride, models,
                         model_row, data_row, grads, workspace, workspace_elems, M, stream);
}

extern "C" int cfa_ge_grad_2nn_rows_f32(const float* x, const float* y, int B, int L, int hidden,
                                        int classes, const float* models, const int32_t* model_row,
                                        const int32_t* data_row, float* grads, float* workspace,
                                        size_t workspace_elems, int M, void* stream) {
  if (M > 0 && (!model_row || !data_row))
    return fail(CFA_E_INVALID, "cfa_ge_grad_2nn_rows_f32: null row table");
  return launch_grad_2nn("cfa_ge_grad_2nn_rows_f32", x, y, B, L, hidden, classes, models, model_row, data_row,
                         grads, workspace, workspace_elems, M, stream);
}
