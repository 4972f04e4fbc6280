/* C-ABI demo: drives libcfa.so from plain C (no Python, no torch) through include/cfa_engine.h.
 * Mixes a local bucket with N neighbour buckets (TF2 rule, eps = 1/(N+1), consensus_v3.py:145,
 * 153-155), then checks the result against a CPU evaluation of the same fp32 chain, bit for bit.
 * Also exercises the FedAvg divisor form and the error path. Exit status 0 = pass. */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cfa_engine.h"

#define CHECK_HIP(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 2; } } while (0)

static unsigned lcg(unsigned* s) { *s = *s * 1664525u + 1013904223u; return *s; }

int main(void) {
  enum { N = 4 };
  const size_t P = 1000003;
  float* h[N + 1];
  float* d[N + 1];
  unsigned seed = 12345u;
  for (int k = 0; k <= N; ++k) {
    h[k] = (float*)malloc(P * sizeof(float));
    for (size_t i = 0; i < P; ++i) h[k][i] = (float)((int)(lcg(&seed) >> 9) - (1 << 22)) / (float)(1 << 20);
    CHECK_HIP(hipMalloc((void**)&d[k], P * sizeof(float)));
    CHECK_HIP(hipMemcpy(d[k], h[k], P * sizeof(float), hipMemcpyHostToDevice));
  }
  float* d_out;
  CHECK_HIP(hipMalloc((void**)&d_out, P * sizeof(float)));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));

  const float* nbrs[N] = {d[1], d[2], d[3], d[4]};
  float alphas[N];
  for (int j = 0; j < N; ++j) alphas[j] = 1.0f / (N + 1);
  if (cfa_mix_seq_f32(d_out, d[0], nbrs, alphas, N, P, (void*)st) != CFA_OK) {
    fprintf(stderr, "cfa_mix_seq_f32: %s\n", cfa_last_error());
    return 1;
  }
  float* out = (float*)malloc(P * sizeof(float));
  CHECK_HIP(hipStreamSynchronize(st));
  CHECK_HIP(hipMemcpy(out, d_out, P * sizeof(float), hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < P; ++i) {
    volatile float w = h[0][i];  /* same three fp32 roundings per step as the kernel */
    for (int j = 0; j < N; ++j) { volatile float t = h[j + 1][i] - w; t = alphas[j] * t; w = w + t; }
    if (memcmp((const void*)&w, &out[i], sizeof(float)) != 0) ++bad;
  }
  /* FedAvg form: p <- p + (u * (x - p)) / C */
  float divs[N] = {4.0f, 4.0f, 4.0f, 4.0f}, us[N] = {1.0f, 1.0f, 1.0f, 1.0f};
  if (cfa_mix_seq_div_f32(d_out, d[0], nbrs, us, divs, N, P, (void*)st) != CFA_OK) return 1;
  CHECK_HIP(hipStreamSynchronize(st));
  CHECK_HIP(hipMemcpy(out, d_out, P * sizeof(float), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < P; ++i) {
    volatile float w = h[0][i];
    for (int j = 0; j < N; ++j) { volatile float t = h[j + 1][i] - w; t = us[j] * t; t = t / divs[j]; w = w + t; }
    if (memcmp((const void*)&w, &out[i], sizeof(float)) != 0) ++bad;
  }
  /* error path: output aliasing a neighbour is rejected with a message */
  int rc = cfa_mix_seq_f32(d[1], d[0], nbrs, alphas, N, P, (void*)st);
  printf("cfa_version=%d mismatches=%zu error_rc=%d error='%s'\n", cfa_version(), bad, rc, cfa_last_error());
  for (int k = 0; k <= N; ++k) { hipFree(d[k]); free(h[k]); }
  hipFree(d_out);
  free(out);
  hipStreamDestroy(st);
  return (bad == 0 && rc == CFA_E_INVALID) ? 0 : 1;
}
