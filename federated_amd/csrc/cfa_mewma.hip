// cfa_mewma.hip — CFA-GE gradient-bucket update on fp32 buckets (MEWMA filter + SGD step with the
// neighbours' gradients), TF1/consensus/cfa_ge_2stage.py:329-371 and :593-621.
#include <utility>

#include "cfa_internal.h"

namespace {

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

// Contiguous case: float4 per lane, g and s streamed once each. The fan-in N is a template
// parameter, so every g and s load of a vector is issued before the first update uses it.
template <int N>
__global__ __launch_bounds__(kBlock) void mewma_vec_kernel(MewmaArgs a, long long nvec) {
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec;
       i += (long long)gridDim.x * kBlock) {
    f4 W = ld4<false>(a.W, i);  // W and s are rewritten in place: default policy (see compress)
    f4 g[N], s_old[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      g[j] = ld4<true>(a.g[j], i);
      if (!a.init) s_old[j] = ld4<false>(a.s[j], i);
    }
    const long long e0 = i * 4;
    f4 lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) lr[c] = (e0 + c) < a.split ? a.lr1 : a.lr2;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      f4 s;
      if (a.init) {
        s = g[j];
      } else {
        s = a.rho * g[j] + a.one_minus_rho * s_old[j];  // numpy: rho*g + (1-rho)*s
      }
      st4<false>(a.s[j], i, s);
      W = W - lr * (a.filtered ? s : g[j]);
    }
    st4<false>(a.W, i, W);
  }
}

template <int... Ns>
static void launch_mewma_vec(int m, unsigned grid, hipStream_t st, const MewmaArgs& a, long long nvec,
                             std::integer_sequence<int, Ns...>) {
  ((m == Ns + 1 ? (void)(mewma_vec_kernel<Ns + 1><<<grid, kBlock, 0, st>>>(a, nvec)) : (void)0), ...);
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

}  // namespace

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
        // one workgroup per CU: 0.792 against 0.778 of peak on the same buffers
        // (tools/kernel_rooflines.py --bpc-variants)
        launch_mewma_vec(m, grid_for_own((nvec + kBlock - 1) / kBlock, 1), st, a, nvec,
                         std::make_integer_sequence<int, CFA_MAX_FANIN>{});
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

