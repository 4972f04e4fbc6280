// Host-side AddressSanitizer / UBSan fuzz harness for the MQTT payload codec
// (federated_amd/csrc/cfa_payload.cpp). Built and run by tools/asan/run_payload_fuzz.sh on the CPU:
// mutates seed payloads (files given on the command line), parses them and reads every key.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char*) {}

static void exercise(const std::vector<unsigned char>& b) {
  cfa_payload_t* h = nullptr;
  if (cfa_payload_parse(b.data(), b.size(), &h) != CFA_OK) return;
  const int nk = cfa_payload_num_keys(h);
  for (int i = 0; i < nk; ++i) {
    const char* k;
    size_t len;
    if (cfa_payload_key(h, i, &k, &len) != CFA_OK) continue;
    std::string key(k, len);
    int kind, ndim;
    int64_t shape[CFA_PAYLOAD_MAX_DIM], numel;
    if (cfa_payload_info(h, key.c_str(), &kind, &ndim, shape, &numel) != CFA_OK) continue;
    int64_t iv;
    double fv;
    cfa_payload_scalar(h, key.c_str(), &kind, &iv, &fv);
    if (numel >= 0 && numel < (1 << 24)) {
      std::vector<double> d((size_t)numel + 1);
      std::vector<float> f((size_t)numel + 1);
      cfa_payload_read_f64(h, key.c_str(), d.data(), numel);
      cfa_payload_read_f32(h, key.c_str(), f.data(), numel);
    }
  }
  cfa_payload_free(h);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10000;
  std::mt19937_64 rng(12345);
  long parsed = 0;
  for (int a = 2; a < argc; ++a) {
    FILE* fp = fopen(argv[a], "rb");
    if (!fp) return 2;
    std::vector<unsigned char> seed;
    int c;
    while ((c = fgetc(fp)) != EOF) seed.push_back((unsigned char)c);
    fclose(fp);
    exercise(seed);
    for (int it = 0; it < iters; ++it) {
      std::vector<unsigned char> b = seed;
      const int flips = 1 + (int)(rng() % 4);
      for (int q = 0; q < flips; ++q) b[rng() % b.size()] = (unsigned char)rng();
      if (rng() % 8 == 0) b.resize(rng() % (b.size() + 1));  // truncation
      exercise(b);
      ++parsed;
    }
    // encode round trip of a float array under the sanitizers
    std::vector<float> w(70000);
    for (size_t i = 0; i < w.size(); ++i) w[i] = (float)i * 0.5f;
    int64_t shp[2] = {350, 200};
    cfa_payload_item_t items[2] = {{"model_layer0", CFA_PAYLOAD_F32_ARRAY, w.data(), 2, shp, 0, 0},
                                   {"device", CFA_PAYLOAD_INT, nullptr, 0, nullptr, 3, 0}};
    size_t n = 0;
    if (cfa_payload_encode(items, 2, 4, nullptr, 0, &n) != CFA_OK) return 3;
    std::vector<unsigned char> out(n);
    if (cfa_payload_encode(items, 2, 4, out.data(), out.size(), &n) != CFA_OK) return 4;
    exercise(out);
  }
  printf("payload fuzz: %ld mutated payloads parsed under ASan/UBSan, no finding\n", parsed);
  return 0;
}
