// Phase timing probe for the population form of the CFA-GE gradient launch at config 3
// (32 evaluations = 16 devices x 2 neighbours, 24 samples, batch split over grid.y): prints the
// phases of workgroup (0, 0) and the spread of every workgroup's start and end stamps over the
// launch (dispatch skew vs per-workgroup latency). Build and run: tools/probe/run_grad_phases.sh
#define CFA_GRAD_PHASES 1
#include "../../federated_amd/csrc/cfa_grad.hip"

#include <algorithm>
#include <vector>

extern "C" void cfa_internal_set_error(const char*) {}

static void report(const char* name, int first, int last, int nwg, int clk) {
  unsigned long long ph[32];
  static unsigned long long wg[4096][2];
  hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_phase), sizeof(ph));
  hipMemcpyFromSymbol(wg, HIP_SYMBOL(g_wg), sizeof(wg));
  const double us = 1000.0 / clk;
  printf("%s wg(0,0) phases (us):", name);
  for (int k = first + 1; k <= last; ++k) printf(" p%d=%.2f", k, (double)(ph[k] - ph[k - 1]) * us);
  printf(" total=%.2f\n", (double)(ph[last] - ph[first]) * us);
  unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
  double dur = 0, dmax = 0;
  for (int i = 0; i < nwg; ++i) {
    s0 = std::min(s0, wg[i][0]), s1 = std::max(s1, wg[i][0]);
    e0 = std::min(e0, wg[i][1]), e1 = std::max(e1, wg[i][1]);
    const double d = (double)(wg[i][1] - wg[i][0]) * us;
    dur += d, dmax = std::max(dmax, d);
  }
  printf("%s %d workgroups: starts spread %.2f us, first start -> last end %.2f us, per-wg mean %.2f max %.2f us\n",
         name, nwg, (double)(s1 - s0) * us, (double)(e1 - s0) * us, dur / nwg, dmax);
}

int main() {
  const int D = 16, N = 2, M = D * N, B = 24, L = 512, C = 8;
  const int Pc = 16 * 8 + 8 + 21 * 8 * C + C, Pn = L * 32 + 32 + 32 * C + C;
  std::vector<float> hx((size_t)D * B * L), hy((size_t)D * B * C, 0.f), hm((size_t)D * Pn);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
  for (int i = 0; i < D * B; ++i) hy[(size_t)i * C + i % C] = 1.f;
  for (size_t i = 0; i < hm.size(); ++i) hm[i] = (float)((i * 40503u) % 1000) / 5000.f - 0.1f;
  std::vector<int> mrow(M), drow(M);
  for (int i = 0; i < D; ++i)
    for (int n = 0; n < N; ++n) mrow[i * N + n] = (i + 1 + n) % D, drow[i * N + n] = i;
  float *x, *y, *m, *g, *ws;
  int *mr, *dr;
  hipMalloc(&x, hx.size() * 4);
  hipMalloc(&y, hy.size() * 4);
  hipMalloc(&m, hm.size() * 4);
  hipMalloc(&g, (size_t)M * Pn * 4);
  const size_t wsn = std::max(cfa_ge_grad_workspace_elems(M, B, Pc), cfa_ge_grad_workspace_elems(M, B, Pn));
  hipMalloc(&ws, std::max<size_t>(wsn, 1) * 4);
  hipMemset(ws, 0, std::max<size_t>(wsn, 1) * 4);  // the split launch's arrival counters start at zero
  hipMalloc(&mr, M * 4);
  hipMalloc(&dr, M * 4);
  hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(y, hy.data(), hy.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(m, hm.data(), hm.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(mr, mrow.data(), M * 4, hipMemcpyHostToDevice);
  hipMemcpy(dr, drow.data(), M * 4, hipMemcpyHostToDevice);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0);  // kHz
  for (int kind = 0; kind < 2; ++kind) {
    const int P = kind == 0 ? Pc : Pn;
    const int sp = (int)(cfa_ge_grad_workspace_elems(M, B, P) / ((size_t)M * P));
    for (int rep = 0; rep < 5; ++rep) {
      int rc = kind == 0 ? cfa_ge_grad_cnn_rows_f32(x, y, B, L, C, 16, 8, 5, m, mr, dr, g, ws, wsn, M, nullptr)
                         : cfa_ge_grad_2nn_rows_f32(x, y, B, L, 32, C, m, mr, dr, g, ws, wsn, M, nullptr);
      hipDeviceSynchronize();
      if (rc) {
        printf("rc %d\n", rc);
        return 1;
      }
    }
    char name[64];
    snprintf(name, sizeof(name), "%s split %d", kind == 0 ? "cnn" : "2nn", std::max(sp, 1));
    report(name, kind == 0 ? 0 : 10, kind == 0 ? 8 : 17, M * std::max(sp, 1), clk);
  }
  return 0;
}
