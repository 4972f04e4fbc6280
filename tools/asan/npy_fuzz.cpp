// Host-side AddressSanitizer / UBSan fuzz harness for the numpy .npy / .npz reader
// (federated_amd/csrc/cfa_npy.cpp). Built and run by tools/asan/run_npy_fuzz.sh on the CPU:
// mutates seed files (given on the command line) in memory, parses them with cfa_npy_parse and
// touches every array's bytes; the seeds are also read from disk with cfa_npy_read.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char*) {}

static long exercise(const std::vector<unsigned char>& b) {
  // a private copy sized exactly, so reads past the image are caught
  unsigned char* img = b.empty() ? nullptr : static_cast<unsigned char*>(malloc(b.size()));
  for (size_t i = 0; i < b.size(); ++i) img[i] = b[i];
  cfa_npy_t* h = nullptr;
  long sum = 0;
  if (cfa_npy_parse(img, b.size(), &h) == CFA_OK) {
    const int n = cfa_npy_num_arrays(h);
    const cfa_npy_array_t* a = cfa_npy_arrays(h);
    for (int i = 0; i < n; ++i) {
      if (a[i].ndim < 0 || a[i].ndim > CFA_NPY_MAX_DIM) exit(3);
      const unsigned char* d = static_cast<const unsigned char*>(a[i].data);
      for (size_t k = 0; k < a[i].nbytes; ++k) sum += d[k];
      for (const char* c = a[i].descr; *c; ++c) sum += *c;
      if (a[i].name)
        for (const char* c = a[i].name; *c; ++c) sum += *c;
    }
    sum += cfa_npy_kind(h) + 1;
    cfa_npy_free(h);
  }
  free(img);
  return sum;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10000;
  std::mt19937_64 rng(4242);
  long parsed = 0, ok = 0;
  for (int a = 2; a < argc; ++a) {
    cfa_npy_t* h = nullptr;
    if (cfa_npy_read(argv[a], &h) != CFA_OK) return 4;  // every seed must read
    cfa_npy_free(h);
    FILE* fp = fopen(argv[a], "rb");
    if (!fp) return 2;
    std::vector<unsigned char> seed;
    int c;
    while ((c = fgetc(fp)) != EOF) seed.push_back((unsigned char)c);
    fclose(fp);
    if (!exercise(seed)) return 5;
    for (int it = 0; it < iters; ++it) {
      std::vector<unsigned char> b = seed;
      const int flips = 1 + (int)(rng() % 5);
      for (int q = 0; q < flips; ++q) {
        const size_t at = (rng() % 4 == 0) ? rng() % std::min<size_t>(b.size(), 512) : rng() % b.size();
        b[at] = (unsigned char)rng();  // a quarter of the flips hit the header / pickle opcodes
      }
      if (rng() % 5 == 0) b.resize(rng() % (b.size() + 1));  // truncation
      ok += exercise(b) != 0;
      ++parsed;
    }
  }
  printf("npy fuzz: %ld mutated files parsed under ASan/UBSan (%ld accepted), no finding\n", parsed, ok);
  return 0;
}
