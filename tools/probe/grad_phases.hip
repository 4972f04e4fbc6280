// Phase timing probe for the CFA-GE gradient kernels: builds csrc/cfa_grad.hip with
// CFA_GRAD_PHASES (wall_clock64 stamps after each barrier of workgroup 0) and prints the time of
// every phase at the driver's shapes. Build: tools/probe/run_grad_phases.sh
#define CFA_GRAD_PHASES 1
#include "../../federated_amd/csrc/cfa_grad.hip"

#include <vector>

extern "C" void cfa_internal_set_error(const char*) {}

int main() {
  const int B = 24, L = 512, C = 8, M = 2;
  std::vector<float> hx(B * L), hy(B * C, 0.f), hm(M * 16680);
  for (size_t i = 0; i < hx.size(); ++i) hx[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
  for (int b = 0; b < B; ++b) hy[b * C + b % C] = 1.f;
  for (size_t i = 0; i < hm.size(); ++i) hm[i] = (float)((i * 40503u) % 1000) / 5000.f - 0.1f;
  float *x, *y, *m, *g;
  hipMalloc(&x, hx.size() * 4);
  hipMalloc(&y, hy.size() * 4);
  hipMalloc(&m, hm.size() * 4);
  hipMalloc(&g, hm.size() * 4);
  hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(y, hy.data(), hy.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(m, hm.data(), hm.size() * 4, hipMemcpyHostToDevice);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeWallClockRate, 0);  // kHz
  for (int kind = 0; kind < 2; ++kind) {
    for (int rep = 0; rep < 3; ++rep) {
      int rc = kind == 0 ? cfa_ge_grad_cnn_f32(x, y, B, L, C, 16, 8, 5, m, g, M, nullptr)
                         : cfa_ge_grad_2nn_f32(x, y, B, L, 32, C, m, g, M, nullptr);
      hipDeviceSynchronize();
      if (rc) { printf("rc %d\n", rc); return 1; }
    }
    unsigned long long ph[32];
    hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_phase), sizeof(ph));
    const int first = kind == 0 ? 0 : 10, last = kind == 0 ? 8 : 17;
    printf("%s kernel phases (us):", kind == 0 ? "cnn" : "2nn");
    for (int k = first + 1; k <= last; ++k) printf(" p%d=%.2f", k, (double)(ph[k] - ph[k - 1]) * 1000.0 / clk);
    printf(" total=%.2f\n", (double)(ph[last] - ph[first]) * 1000.0 / clk);
  }
  return 0;
}
