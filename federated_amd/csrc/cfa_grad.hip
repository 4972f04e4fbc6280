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

__host__ __device__ inline int same_left(int L, int k, int s) {
  const int out = (L + s - 1) / s;
  const int total = max((out - 1) * s + k - L, 0);
  return total / 2;
}

// Softmax + clipped cross-entropy backward for one sample: logits[C] in, dlogits[C] out (in place).
// d cost / d pred_c = -(y_c / clip(pred_c)) / B where the clip passes the gradient; then the
// softmax gradient (dp - sum(dp * p)) * p (TF SoftmaxGrad).
__device__ void softmax_xent_backward(float* z, const float* y, int C, float invB) {
  float mx = z[0];
  for (int c = 1; c < C; ++c) mx = fmaxf(mx, z[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) {
    z[c] = expf(z[c] - mx);
    s += z[c];
  }
  auto dpred = [&](float p, int c) {
    const bool pass = p >= kClipLo && p <= kClipHi;
    return pass ? -(y[c] / fminf(fmaxf(p, kClipLo), kClipHi)) * invB : 0.f;
  };
  float dot = 0.f;
  for (int c = 0; c < C; ++c) {
    z[c] = z[c] / s;  // pred
    dot = fmaf(dpred(z[c], c), z[c], dot);
  }
  for (int c = 0; c < C; ++c) z[c] = (dpred(z[c], c) - dot) * z[c];
}

struct CnnDims {
  int B, L, C, F, NC, S;
  int L1, L2, pl, ql;  // conv / pool output lengths, left pads
  int Bc;              // samples per LDS-resident chunk
  long long P;         // parameters per model
};

// Gradient sums run over all B samples; samples go through LDS in chunks of Bc. Each output
// element is owned by one thread for the whole launch (the same index loop every chunk), so the
// per-chunk partial sums accumulate in the output bucket without atomics, in a fixed order.
__global__ __launch_bounds__(kBlock) void grad_cnn_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ y,
                                                          const float* __restrict__ models,
                                                          float* __restrict__ grads, CnnDims d) {
  extern __shared__ float lds[];
  const int LN = d.L2 * d.NC;
  float* W1 = lds;                        // [F][NC]
  float* b1 = W1 + d.F * d.NC;            // [NC]
  float* W2 = b1 + d.NC;                  // [LN][C]
  float* b2 = W2 + LN * d.C;              // [C]
  float* pooled = b2 + d.C;               // [Bc][L2][NC]
  int* arg = reinterpret_cast<int*>(pooled + d.Bc * LN);  // conv position of each window's max
  float* dfc = reinterpret_cast<float*>(arg + d.Bc * LN); // [Bc][LN]
  float* zl = dfc + d.Bc * LN;            // [Bc][C]: logits, then d logits
  const float* m = models + (long long)blockIdx.x * d.P;
  float* g = grads + (long long)blockIdx.x * d.P;
  const int tid = threadIdx.x, T = blockDim.x;
  const int nW1 = d.F * d.NC, nW2 = LN * d.C;
  float* gW1 = g;
  float* gb1 = gW1 + nW1;
  float* gW2 = gb1 + d.NC;
  float* gb2 = gW2 + nW2;
  const float invB = 1.0f / (float)d.B;

  for (int i = tid; i < nW1 + d.NC + nW2 + d.C; i += T) W1[i] = m[i];  // model bucket = W1 b1 W2 b2
  __syncthreads();

  for (int b0 = 0; b0 < d.B; b0 += d.Bc) {
    const int nb = min(d.Bc, d.B - b0);
    const float* xc = x + (long long)b0 * d.L;
    const float* yc = y + (long long)b0 * d.C;
    const bool first = b0 == 0;
    // conv + bias + relu evaluated inside each pooling window; keep the max and its position
    for (int idx = tid; idx < nb * LN; idx += T) {
      const int b = idx / LN, r = idx % LN, q = r / d.NC, c = r % d.NC;
      float best = -INFINITY;
      int barg = -1;
      for (int j = 0; j < d.S; ++j) {
        const int p = q * d.S - d.ql + j;
        if (p < 0 || p >= d.L1) continue;
        float z = 0.f;
        for (int k = 0; k < d.F; ++k) {
          const int t = p * d.S + k - d.pl;
          if (t >= 0 && t < d.L) z = fmaf(xc[b * d.L + t], W1[k * d.NC + c], z);
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
    for (int idx = tid; idx < nb * d.C; idx += T) {  // logits
      const int b = idx / d.C, k = idx % d.C;
      float z = 0.f;
      for (int i = 0; i < LN; ++i) z = fmaf(pooled[b * LN + i], W2[i * d.C + k], z);
      zl[idx] = z + b2[k];
    }
    __syncthreads();
    for (int b = tid; b < nb; b += T) softmax_xent_backward(zl + b * d.C, yc + b * d.C, d.C, invB);
    __syncthreads();

    // dense layer gradients and the gradient flowing into the pooled features
    for (int idx = tid; idx < nW2; idx += T) {
      const int i = idx / d.C, k = idx % d.C;
      float s = first ? 0.f : gW2[idx];
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

    // conv gradients: only each window's max position receives gradient (windows do not overlap)
    for (int idx = tid; idx < nW1 + d.NC; idx += T) {
      if (idx < nW1) {
        const int k = idx / d.NC, c = idx % d.NC;
        float s = first ? 0.f : gW1[idx];
        for (int b = 0; b < nb; ++b)
          for (int q = 0; q < d.L2; ++q) {
            const int e = b * LN + q * d.NC + c;
            const float gz = dfc[e];
            const int t = arg[e] * d.S + k - d.pl;
            if (gz != 0.f && t >= 0 && t < d.L) s = fmaf(gz, xc[b * d.L + t], s);
          }
        gW1[idx] = s;
      } else {
        const int c = idx - nW1;
        float s = first ? 0.f : gb1[c];
        for (int b = 0; b < nb; ++b)
          for (int q = 0; q < d.L2; ++q) s += dfc[b * LN + q * d.NC + c];
        gb1[c] = s;
      }
    }
    __syncthreads();  // the chunk's LDS is reused by the next one
  }
}

struct NnDims {
  int B, L, H, C;
  int Bc;
  long long P;
};

__global__ __launch_bounds__(kBlock) void grad_2nn_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ y,
                                                          const float* __restrict__ models,
                                                          float* __restrict__ grads, NnDims d) {
  extern __shared__ float lds[];
  float* b1 = lds;                 // [H]
  float* W2 = b1 + d.H;            // [H][C]
  float* b2 = W2 + d.H * d.C;      // [C]
  float* act = b2 + d.C;           // [Bc][H] relu(x W1 + b1)
  float* dz = act + d.Bc * d.H;    // [Bc][H]
  float* zl = dz + d.Bc * d.H;     // [Bc][C]
  const long long nW1 = (long long)d.L * d.H;
  const float* m = models + (long long)blockIdx.x * d.P;
  const float* W1 = m;             // [L][H], read from global (L2-resident)
  float* g = grads + (long long)blockIdx.x * d.P;
  float* gW1 = g;
  float* gb1 = gW1 + nW1;
  float* gW2 = gb1 + d.H;
  float* gb2 = gW2 + d.H * d.C;
  const int tid = threadIdx.x, T = blockDim.x;
  const float invB = 1.0f / (float)d.B;

  for (int i = tid; i < d.H + d.H * d.C + d.C; i += T) b1[i] = m[nW1 + i];
  __syncthreads();
  for (int b0 = 0; b0 < d.B; b0 += d.Bc) {
    const int nb = min(d.Bc, d.B - b0);
    const float* xc = x + (long long)b0 * d.L;
    const float* yc = y + (long long)b0 * d.C;
    const bool first = b0 == 0;
    for (int idx = tid; idx < nb * d.H; idx += T) {
      const int b = idx / d.H, h = idx % d.H;
      float z = 0.f;
      for (int i = 0; i < d.L; ++i) z = fmaf(xc[b * d.L + i], W1[(long long)i * d.H + h], z);
      z += b1[h];
      act[idx] = z > 0.f ? z : 0.f;
    }
    __syncthreads();
    for (int idx = tid; idx < nb * d.C; idx += T) {
      const int b = idx / d.C, k = idx % d.C;
      float z = 0.f;
      for (int h = 0; h < d.H; ++h) z = fmaf(act[b * d.H + h], W2[h * d.C + k], z);
      zl[idx] = z + b2[k];
    }
    __syncthreads();
    for (int b = tid; b < nb; b += T) softmax_xent_backward(zl + b * d.C, yc + b * d.C, d.C, invB);
    __syncthreads();
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
    for (long long idx = tid; idx < nW1; idx += T) {  // consecutive lanes: consecutive h (coalesced)
      const int i = (int)(idx / d.H), h = (int)(idx % d.H);
      float s = first ? 0.f : gW1[idx];
      for (int b = 0; b < nb; ++b) s = fmaf(xc[b * d.L + i], dz[b * d.H + h], s);
      gW1[idx] = s;
    }
    for (int h = tid; h < d.H; h += T) {
      float s = first ? 0.f : gb1[h];
      for (int b = 0; b < nb; ++b) s += dz[b * d.H + h];
      gb1[h] = s;
    }
    __syncthreads();
  }
}

// Dynamic LDS per workgroup: the device limit, capped at 64 KiB (the default dynamic-LDS bound of
// a kernel without a raised attribute); larger sample counts run in chunks.
int lds_limit() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 65536;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || v <= 0)
    return 65536;
  return std::min(v, 65536);
}

}  // namespace

extern "C" int cfa_ge_grad_cnn_f32(const float* x, const float* y, int B, int L, int classes,
                                   int filter, int number, int stride, const float* models,
                                   float* grads, int M, void* stream) {
  if (M < 0 || B < 1 || L < 1 || classes < 1 || filter < 1 || number < 1 || stride < 1)
    return fail(CFA_E_INVALID, "cfa_ge_grad_cnn_f32: bad dimensions (B %d L %d C %d F %d NC %d S %d M %d)",
                B, L, classes, filter, number, stride, M);
  if (M == 0) return CFA_OK;
  if (!x || !y || !models || !grads) return fail(CFA_E_INVALID, "cfa_ge_grad_cnn_f32: null buffer");
  CnnDims d;
  d.B = B, d.L = L, d.C = classes, d.F = filter, d.NC = number, d.S = stride;
  d.L1 = (L + stride - 1) / stride;
  d.L2 = (d.L1 + stride - 1) / stride;
  d.pl = same_left(L, filter, stride);
  d.ql = same_left(d.L1, stride, stride);
  const long long LN = (long long)d.L2 * number;
  d.P = (long long)filter * number + number + LN * classes + classes;
  const long long fixed = 4LL * (d.F * d.NC + d.NC + LN * d.C + d.C);
  const long long per_sample = 4LL * (3LL * LN + d.C);
  const long long room = (long long)lds_limit() - fixed;
  if (room < per_sample)
    return fail(CFA_E_UNSUPPORTED, "cfa_ge_grad_cnn_f32: the model alone needs %lld bytes of LDS", fixed);
  d.Bc = (int)std::min<long long>(B, room / per_sample);
  const long long lds = fixed + per_sample * d.Bc;
  grad_cnn_kernel<<<M, kBlock, (size_t)lds, static_cast<hipStream_t>(stream)>>>(x, y, models, grads, d);
  return check_launch("grad_cnn_kernel");
}

extern "C" int cfa_ge_grad_2nn_f32(const float* x, const float* y, int B, int L, int hidden,
                                   int classes, const float* models, float* grads, int M,
                                   void* stream) {
  if (M < 0 || B < 1 || L < 1 || hidden < 1 || classes < 1)
    return fail(CFA_E_INVALID, "cfa_ge_grad_2nn_f32: bad dimensions (B %d L %d H %d C %d M %d)", B, L, hidden,
                classes, M);
  if (M == 0) return CFA_OK;
  if (!x || !y || !models || !grads) return fail(CFA_E_INVALID, "cfa_ge_grad_2nn_f32: null buffer");
  NnDims d;
  d.B = B, d.L = L, d.H = hidden, d.C = classes;
  d.P = (long long)L * hidden + hidden + (long long)hidden * classes + classes;
  const long long fixed = 4LL * (hidden + (long long)hidden * classes + classes);
  const long long per_sample = 4LL * (2LL * hidden + classes);
  const long long room = (long long)lds_limit() - fixed;
  if (room < per_sample)
    return fail(CFA_E_UNSUPPORTED, "cfa_ge_grad_2nn_f32: the model alone needs %lld bytes of LDS", fixed);
  d.Bc = (int)std::min<long long>(B, room / per_sample);
  const long long lds = fixed + per_sample * d.Bc;
  grad_2nn_kernel<<<M, kBlock, (size_t)lds, static_cast<hipStream_t>(stream)>>>(x, y, models, grads, d);
  return check_launch("grad_2nn_kernel");
}
