// cfa_population.hip — whole-population rounds: the CSR one-launch kernel
// (cfa_mix_population_f32) and the sliding-window passes (cfa_mix_window_f32) that load each
// row of a ring window once for up to 8 consecutive devices.
#include "cfa_internal.h"

// Resident workgroups per CU across a whole population launch (all devices together). 8 by
// default; CFA_POP_WG_PER_CU overrides it per call (read at each launch, so one process can
// compare values: tools/probe/pop_shape.py).
static int pop_wg_per_cu() {
  const char* s = getenv("CFA_POP_WG_PER_CU");
  const int v = s ? atoi(s) : 0;
  return v > 0 ? v : 8;
}

namespace {

// ------------------------------------------------------------------------------------------
// Population round: grid.y = device, grid.x = tiles. CSR lists each device's sources.
// ------------------------------------------------------------------------------------------
template <int RULE>
__global__ __launch_bounds__(kBlock) void population_kernel(float* const* out_ptrs,
                                                            const float* const* src_ptrs,
                                                            const int32_t* csr_ptr,
                                                            const int32_t* csr_idx,
                                                            const float* csr_coef,
                                                            long long nvec, long long P) {
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
  // the < 4-element tail, in the same launch (one kernel boundary fewer per round): the
  // scalar form of the same operations, so every element rounds as in the float4 body
  if (blockIdx.x == 0 && nvec * 4 + threadIdx.x < P) {
    const long long i = nvec * 4 + threadIdx.x;
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
    out[i] = w;
  }
}

// TF1 population round (cfa_mix_population_tf1_f32): per device the numpy-2 chain of the TF1
// modules (cfa.py:66-76): the first subtraction x_1 - w of two fp32 arrays is fp32, every later
// operation fp64 with the fp64 coefficients eps * wf_j, one rounding to fp32 at the end. A TF1
// driver assigns the returned fp64 arrays into its fp32 TF variables, so fp32 buckets mixed this
// way follow the reference run's trajectory exactly. Same operations as cfa_mix_tf1_f32.
__global__ __launch_bounds__(kBlock) void population_tf1_kernel(float* const* out_ptrs,
                                                                const float* const* src_ptrs,
                                                                const int32_t* csr_ptr,
                                                                const int32_t* csr_idx,
                                                                const double* csr_coef,
                                                                long long nvec, long long P,
                                                                CompressParams cp) {
  const int d = blockIdx.y;
  const int e0 = csr_ptr[d], e1 = csr_ptr[d + 1];
  float* out = out_ptrs[d];
  const float* l = src_ptrs[csr_idx[e0]];
  unsigned kept = 0;
  // the compression epilogue (cfa_ongraphs.py:225-273) on [cbegin, cend): fp64 against the
  // pre-mix local after a mix, fp32 on the local itself for a device without neighbours (the
  // reference then compresses the caller's fp32 array in place, numpy-2 fp32 thresholds)
  auto epi = [&](double w, float lv, long long e) -> float {
    if (cp.mode && e >= cp.cbegin && e < cp.cend) return (float)compress_one_d(w, (double)lv, cp, kept);
    return (float)w;
  };
  auto epi0 = [&](float lv, long long e) -> float {
    if (cp.mode && e >= cp.cbegin && e < cp.cend) return compress_one(lv, lv, cp, kept);
    return lv;
  };
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long long)gridDim.x * kBlock) {
    const f4 lv = ld4<true>(l, i);
    f4 y;
    if (e1 - e0 <= 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) y[c] = epi0(lv[c], 4 * i + c);
    } else {
      const f4 x1 = ld4<true>(src_ptrs[csr_idx[e0 + 1]], i);
      double w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float dd = x1[c] - lv[c];                      // fp32 - fp32
        w[c] = (double)lv[c] + csr_coef[e0 + 1] * (double)dd;  // fp64 from here on
      }
      for (int e = e0 + 2; e < e1; ++e) {
        const f4 x = ld4<true>(src_ptrs[csr_idx[e]], i);
        const double a = csr_coef[e];
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = w[c] + a * ((double)x[c] - w[c]);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) y[c] = epi(w[c], lv[c], 4 * i + c);
    }
    st4<true>(out, i, y);
  }
  if (blockIdx.x == 0) {  // the < 4-element tail
    for (long long i = nvec * 4 + threadIdx.x; i < P; i += kBlock) {
      const float lv = l[i];
      float y;
      if (e1 - e0 <= 1) {
        y = epi0(lv, i);
      } else {
        const float dd = src_ptrs[csr_idx[e0 + 1]][i] - lv;
        double w = (double)lv + csr_coef[e0 + 1] * (double)dd;
        for (int e = e0 + 2; e < e1; ++e) w = w + csr_coef[e] * ((double)src_ptrs[csr_idx[e]][i] - w);
        y = epi(w, lv, i);
      }
      out[i] = y;
    }
  }
  if (cp.mode) block_add_count(kept, cp.kept + d);
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
__device__ __forceinline__ void window_body(const WindowArgs& w, long long nvec) {
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

template <int HL, int HR, int U, bool SC1>
__global__ __launch_bounds__(kBlock) void window_vec_kernel(WindowArgs w, long long nvec) {
  window_body<HL, HR, U, SC1>(w, nvec);
}

// A whole ring-window round of a stacked population in ONE launch (cfa_mix_ring_round_f32):
// grid.y = pass p over devices [8p, 8p + nb); each block derives its pass's rows from the stack
// base and pitch (row g of the window = in + ((8p - HL + g) mod D) * pitch), then runs the
// window pass body. Same operations as one cfa_mix_window_f32 launch per pass.
struct RingArgs {
  const float* in;
  float* out;
  const float* alphas;  // [D] device array, one coefficient per device
  long long pitch;      // floats between consecutive devices' rows
  long long off;        // element offset of this launch's chunk
  int D;
};

template <int HL, int HR, int U, bool SC1>
__global__ __launch_bounds__(kBlock) void ring_round_kernel(RingArgs ra, long long nvec) {
  const int p = blockIdx.y;
  WindowArgs w;
  w.nb = min(kWinMaxDev, ra.D - p * kWinMaxDev);
#pragma unroll
  for (int k = 0; k < kWinMaxDev + HL + HR; ++k) {
    const int g = ((p * kWinMaxDev - HL + k) % ra.D + ra.D) % ra.D;
    w.rows[k] = ra.in + (long long)g * ra.pitch + ra.off;
  }
#pragma unroll
  for (int b = 0; b < kWinMaxDev; ++b) {
    const int d = min(p * kWinMaxDev + b, ra.D - 1);
    w.out[b] = ra.out + (long long)d * ra.pitch + ra.off;
    w.a[b] = ra.alphas[d];
  }
  window_body<HL, HR, U, SC1>(w, nvec);
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

}  // namespace

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
template <int HL, int HR>
void launch_ring_round(const RingArgs& ra, long long nvec, hipStream_t st) {
  const WindowTune t = window_tune();
  const cfa_launch_t lc{t.blocks_per_cu, t.vec, 1};
  const unsigned passes = (unsigned)((ra.D + kWinMaxDev - 1) / kWinMaxDev);
  for (long long done = 0; done < nvec; done += kMaxChunkVec) {
    const long long m = (nvec - done) < kMaxChunkVec ? (nvec - done) : kMaxChunkVec;
    RingArgs c = ra;
    c.off = ra.off + done * 4;
    const long long tiles = (m + (long long)kBlock * t.vec - 1) / ((long long)kBlock * t.vec);
    // the launch's blocks over all passes: about blocks_per_cu per CU in all
    long long gx = (grid_for(tiles, lc) + passes - 1) / passes;
    if (gx < 1) gx = 1;
    if (gx > tiles) gx = tiles;
    const dim3 grid((unsigned)gx, passes);
    if (t.vec == 1) {
      if (t.sc1) ring_round_kernel<HL, HR, 1, true><<<grid, kBlock, 0, st>>>(c, m);
      else ring_round_kernel<HL, HR, 1, false><<<grid, kBlock, 0, st>>>(c, m);
    } else {
      if (t.sc1) ring_round_kernel<HL, HR, 2, true><<<grid, kBlock, 0, st>>>(c, m);
      else ring_round_kernel<HL, HR, 2, false><<<grid, kBlock, 0, st>>>(c, m);
    }
  }
}
using RingLaunch = void (*)(const RingArgs&, long long, hipStream_t);
#define CFA_R(L, R) &launch_ring_round<L, R>
const RingLaunch kRingLaunch[5][5] = {
    {CFA_R(0, 0), CFA_R(0, 1), CFA_R(0, 2), CFA_R(0, 3), CFA_R(0, 4)},
    {CFA_R(1, 0), CFA_R(1, 1), CFA_R(1, 2), CFA_R(1, 3), CFA_R(1, 4)},
    {CFA_R(2, 0), CFA_R(2, 1), CFA_R(2, 2), CFA_R(2, 3), CFA_R(2, 4)},
    {CFA_R(3, 0), CFA_R(3, 1), CFA_R(3, 2), CFA_R(3, 3), CFA_R(3, 4)},
    {CFA_R(4, 0), CFA_R(4, 1), CFA_R(4, 2), CFA_R(4, 3), CFA_R(4, 4)}};
#undef CFA_R
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

extern "C" int cfa_mix_ring_round_f32(float* out, const float* in, size_t pitch, const float* alphas, int D,
                                      int hl, int hr, size_t P, void* stream) {
  if (D < 1) return fail(CFA_E_INVALID, "device count %d", D);
  if (hl < 0 || hr < 0 || hl > 4 || hr > 4) return fail(CFA_E_INVALID, "window %d/%d outside 0..4", hl, hr);
  if (hl + hr >= D) return fail(CFA_E_INVALID, "window %d/%d wider than %d devices", hl, hr, D);
  if (!out || !in || !alphas) return fail(CFA_E_INVALID, "null buffer");
  if (pitch < P) return fail(CFA_E_INVALID, "pitch %zu below P %zu", pitch, P);
  if (P == 0) return CFA_OK;
  if ((addr(out) & 15) || (addr(in) & 15) || (pitch % 4) || (P % 4))
    return fail(CFA_E_UNSUPPORTED, "ring round needs 16-byte aligned rows (pitch and P multiples of 4)");
  const long long outb = (long long)addr(out), inb = (long long)addr(in), span = (long long)D * (long long)pitch * 4;
  if (outb < inb + span && inb < outb + span) return fail(CFA_E_INVALID, "out overlaps in");
  if ((long long)(D + kWinMaxDev - 1) / kWinMaxDev > 65535) return fail(CFA_E_INVALID, "D=%d exceeds grid.y", D);
  RingArgs ra{in, out, alphas, (long long)pitch, 0, D};
  kRingLaunch[hl][hr](ra, (long long)(P / 4), (hipStream_t)stream);
  return check_launch("ring_round");
}

extern "C" int cfa_mix_population_tf1_f32(float* const* out_ptrs, const float* const* src_ptrs,
                                          const int32_t* csr_ptr, const int32_t* csr_idx,
                                          const double* csr_coef, int D, size_t P, int mode,
                                          size_t cbegin, size_t cend, unsigned long long* kept_counts,
                                          void* stream) {
  if (D < 0) return fail(CFA_E_INVALID, "negative device count");
  CompressParams cp{};
  if (int rc = compress_params(mode, cp)) return rc;
  if (mode && (!kept_counts || cbegin > cend || cend > P))
    return fail(CFA_E_INVALID, "compression needs per-device counters and a segment within the bucket");
  cp.cbegin = (long long)cbegin;
  cp.cend = (long long)cend;
  cp.kept = kept_counts;
  if (D == 0 || P == 0) return CFA_OK;
  if (!out_ptrs || !src_ptrs || !csr_ptr || !csr_idx || !csr_coef)
    return fail(CFA_E_INVALID, "null population table");
  if (D > 65535) return fail(CFA_E_INVALID, "D=%d exceeds grid.y limit", D);
  const long long nvec = (long long)P / 4;
  long long gx = (nvec + kBlock - 1) / kBlock;
  const long long cap = ((long long)device_cus() * pop_wg_per_cu() + D - 1) / D;
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  population_tf1_kernel<<<dim3((unsigned)gx, (unsigned)D), kBlock, 0, (hipStream_t)stream>>>(
      out_ptrs, src_ptrs, csr_ptr, csr_idx, csr_coef, nvec, (long long)P, cp);
  return check_launch("population_tf1");
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
  // host layer); the body runs on float4, the <4-element tail in the first tile column.
  const long long nvec = (long long)P / 4;
  long long gx = (nvec + 2LL * kBlock - 1) / (2LL * kBlock);
  const long long cap = ((long long)device_cus() * pop_wg_per_cu() + D - 1) / D;
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  dim3 grid((unsigned)gx, (unsigned)D);
  if (rule == CFA_RULE_SEQUENTIAL)
    population_kernel<CFA_RULE_SEQUENTIAL><<<grid, kBlock, 0, st>>>(out_ptrs, src_ptrs, csr_ptr,
                                                                    csr_idx, csr_coef, nvec, (long long)P);
  else
    population_kernel<CFA_RULE_LINEAR><<<grid, kBlock, 0, st>>>(out_ptrs, src_ptrs, csr_ptr,
                                                                csr_idx, csr_coef, nvec, (long long)P);
  if (int rc = check_launch("population")) return rc;
  return CFA_OK;
}


// ------------------------------------------------------------------------------------------
// CFA-GE population step (cfa_ge_population_step_f32): stage-1 mix and the neighbours' gradient
// step of every device in one launch (cfa_ge_2stage.py:446-466 then :591-621). The operations
// and their order are those of cfa_mix_population_f32 followed by cfa_mewma_update_f32, so the
// result is identical to the two launches, minus one write and one read of every mixed model.
// ------------------------------------------------------------------------------------------
namespace {

struct GeStepArgs {
  float* const* out;
  const float* const* src;
  float* const* state;
  const float* const* grad;
  const int32_t* ptr;
  const int32_t* idx;
  const float* coef;
  float rho, one_minus_rho, lr1, lr2;
  long long split;
  int filtered;
  // optional second job of the same launch: sum rsp partial buckets of rM gradient evaluations
  // (rws [rM][rsp][P], written by a partials-only cfa_ge_grad_*_rows_f32) into rout [rM][P]
  const float* rws;
  float* rout;
  int rM, rsp;
};

__device__ __forceinline__ float ge_lr(const GeStepArgs& a, long long i) { return i < a.split ? a.lr1 : a.lr2; }

__global__ __launch_bounds__(kBlock) void ge_step_kernel(GeStepArgs a, long long nvec, long long P) {
  const int d = blockIdx.y;
  if (d >= (int)gridDim.y - a.rM) {  // reduction rows: the split sum in split order (deterministic)
    const long long m = d - ((int)gridDim.y - a.rM);
    const float* w = a.rws + m * a.rsp * P;
    for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < P; i += (long long)gridDim.x * kBlock) {
      float s = w[i];
      for (int sp = 1; sp < a.rsp; ++sp) s += w[(long long)sp * P + i];
      a.rout[m * P + i] = s;
    }
    return;
  }
  const int e0 = a.ptr[d], e1 = a.ptr[d + 1];
  float* out = a.out[d];
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < nvec; i += (long long)gridDim.x * kBlock) {
    f4 w = ld4<false>(a.src[a.idx[e0]], i);
    for (int e = e0 + 1; e < e1; ++e) {  // stage 1: sequential rule
      const f4 x = ld4<false>(a.src[a.idx[e]], i);
      f4 t = x - w;
      t = a.coef[e] * t;
      w = w + t;
    }
    f4 lr;
#pragma unroll
    for (int c = 0; c < 4; ++c) lr[c] = ge_lr(a, i * 4 + c);
    for (int e = e0 + 1; e < e1; ++e) {  // gradient step: MEWMA filter + SGD
      const float* gp = a.grad[e];
      const f4 g = gp ? ld4<false>(gp, i) : f4{0.f, 0.f, 0.f, 0.f};
      const f4 s_old = ld4<false>(a.state[e], i);
      const f4 s = a.rho * g + a.one_minus_rho * s_old;
      st4<false>(a.state[e], i, s);
      w = w - lr * (a.filtered ? s : g);
    }
    st4<false>(out, i, w);
  }
  if (blockIdx.x == 0) {  // the < 4-element tail
    for (long long i = nvec * 4 + threadIdx.x; i < P; i += kBlock) {
      float w = a.src[a.idx[e0]][i];
      for (int e = e0 + 1; e < e1; ++e) {
        float t = a.src[a.idx[e]][i] - w;
        t = a.coef[e] * t;
        w = w + t;
      }
      const float lr = ge_lr(a, i);
      for (int e = e0 + 1; e < e1; ++e) {
        const float g = a.grad[e] ? a.grad[e][i] : 0.f;
        const float t1 = a.rho * g;
        const float t2 = a.one_minus_rho * a.state[e][i];
        const float s = t1 + t2;
        a.state[e][i] = s;
        w = w - lr * (a.filtered ? s : g);
      }
      out[i] = w;
    }
  }
}

}  // namespace

extern "C" int cfa_ge_population_step_f32(float* const* out_ptrs, const float* const* src_ptrs,
                                          float* const* state_ptrs, const float* const* grad_ptrs,
                                          const int32_t* csr_ptr, const int32_t* csr_idx,
                                          const float* csr_coef, int D, double rho, float lr1,
                                          float lr2, size_t lr_split, int use_filtered, size_t P,
                                          const float* reduce_ws, float* reduce_out, int reduce_M,
                                          int reduce_splits, void* stream) {
  if (D < 0) return fail(CFA_E_INVALID, "negative device count");
  if (!reduce_ws) reduce_M = 0;
  if (reduce_M < 0 || (reduce_M > 0 && (!reduce_out || reduce_splits < 1)))
    return fail(CFA_E_INVALID, "bad split reduction (M %d, splits %d)", reduce_M, reduce_splits);
  if ((D == 0 && reduce_M == 0) || P == 0) return CFA_OK;
  if (D > 0 && (!out_ptrs || !src_ptrs || !state_ptrs || !grad_ptrs || !csr_ptr || !csr_idx || !csr_coef))
    return fail(CFA_E_INVALID, "null population table");
  if ((long long)D + reduce_M > 65535) return fail(CFA_E_INVALID, "D + M = %d exceeds grid.y limit", D + reduce_M);
  GeStepArgs a{out_ptrs, src_ptrs, state_ptrs, grad_ptrs, csr_ptr, csr_idx, csr_coef,
               (float)rho, (float)(1.0 - rho), lr1, lr2, (long long)lr_split, use_filtered ? 1 : 0,
               reduce_ws, reduce_out, reduce_M, reduce_splits};
  // buckets are 16-byte aligned (allocator contract, checked by the host layer)
  const long long nvec = (long long)P / 4;
  long long gx = (nvec + kBlock - 1) / kBlock;
  const long long cap = ((long long)device_cus() * pop_wg_per_cu() + D + reduce_M - 1) / (D + reduce_M);
  if (gx > cap) gx = cap;
  if (gx < 1) gx = 1;
  dim3 grid((unsigned)gx, (unsigned)(D + reduce_M));
  ge_step_kernel<<<grid, kBlock, 0, static_cast<hipStream_t>(stream)>>>(a, nvec, (long long)P);
  return check_launch("ge_step_kernel");
}
