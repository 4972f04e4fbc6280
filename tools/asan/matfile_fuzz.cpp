// Host-side AddressSanitizer / UBSan fuzz harness for the MATLAB level-5 codec
// (federated_amd/csrc/cfa_matfile.cpp). Built and run by tools/asan/run_matfile_fuzz.sh on the CPU:
// mutates seed .mat files (given on the command line), reads them back and touches every
// variable's bytes; then writes a file and reads it back under the sanitizers.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char*) {}

static std::vector<unsigned char> slurp(const char* path) {
  std::vector<unsigned char> b;
  FILE* fp = fopen(path, "rb");
  if (!fp) return b;
  int c;
  while ((c = fgetc(fp)) != EOF) b.push_back((unsigned char)c);
  fclose(fp);
  return b;
}

static long exercise(const std::string& path, const std::vector<unsigned char>& b) {
  FILE* fp = fopen(path.c_str(), "wb");
  if (!fp) exit(2);
  fwrite(b.data(), 1, b.size(), fp);
  fclose(fp);
  cfa_mat_t* m = nullptr;
  if (cfa_mat_read(path.c_str(), &m) != CFA_OK) return 0;
  long sum = 0;
  const int n = cfa_mat_num_vars(m);
  const cfa_mat_var_t* v = cfa_mat_vars(m);
  for (int i = 0; i < n; ++i) {
    for (const char* c = v[i].name; *c; ++c) sum += *c;
    const unsigned char* d = static_cast<const unsigned char*>(v[i].data);
    for (size_t k = 0; k < v[i].nbytes; ++k) sum += d[k];
    if (v[i].ndim < 1 || v[i].ndim > CFA_MAT_MAX_DIM) exit(3);
  }
  for (const char* c = cfa_mat_header(m); *c; ++c) sum += *c;
  cfa_mat_free(m);
  return sum + 1;
}

int main(int argc, char** argv) {
  const int iters = argc > 2 ? atoi(argv[2]) : 10000;
  const std::string tmp = argv[1];
  std::mt19937_64 rng(12345);
  long read = 0, ok = 0;
  for (int a = 3; a < argc; ++a) {
    const std::vector<unsigned char> seed = slurp(argv[a]);
    if (seed.empty() || !exercise(tmp, seed)) return 4;  // the seed itself must read
    for (int it = 0; it < iters; ++it) {
      std::vector<unsigned char> b = seed;
      const int flips = 1 + (int)(rng() % 5);
      for (int q = 0; q < flips; ++q) b[rng() % b.size()] = (unsigned char)rng();
      if (rng() % 5 == 0) b.resize(rng() % (b.size() + 1));  // truncation
      ok += exercise(tmp, b) != 0;
      ++read;
    }
  }
  // write + read back under the sanitizers (a 4-byte and a padded variable)
  std::vector<float> w(7 * 5);
  for (size_t i = 0; i < w.size(); ++i) w[i] = (float)i;
  const int32_t s = 3;
  cfa_mat_var_t vars[2] = {{"weights1", 7, 7, 2, {7, 5}, w.data(), w.size() * 4},
                           {"e", 12, 5, 2, {1, 1}, &s, 4}};
  if (cfa_mat_write(tmp.c_str(), "MATLAB 5.0 MAT-file Platform: posix", 2, vars) != CFA_OK) return 5;
  if (!exercise(tmp, slurp(tmp.c_str()))) return 6;
  printf("matfile fuzz: %ld mutated files read under ASan/UBSan (%ld accepted), no finding\n", read, ok);
  return 0;
}
