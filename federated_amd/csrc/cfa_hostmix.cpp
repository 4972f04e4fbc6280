// cfa_hostmix.cpp — the drop-in host path of one CFA mix as a native chunk pipeline
// (host ingress / egress around the mix).
//
// A drop-in call holds its models as per-layer arrays in pageable host memory: the local model
// and n neighbour models (TF2 consensus_v3.py:144-157 mixes the Keras layer lists of the loaded
// .npy files; parameter_server_v2.py:159-161 folds the active devices' models). The GPU reads
// pinned memory over PCIe in place (zero-copy), so the arrays are first packed into pinned
// staging and the result is unpacked from pinned output. Done serially that is pack, then the
// PCIe-bound kernel, then unpack; at the C4 model (VGG-1, 4 neighbours, 21 MB of staging) the
// pack and the kernel cost about the same.
//
// cfa_host_mix_f32 overlaps them: the bucket range is cut into chunks; chunk c of every model is
// packed by a small pool of host threads while the kernel of chunk c - 1 reads its packed slices
// over PCIe; each chunk's result is unpacked into the caller's output layers as soon as its
// kernel is done, while later chunks are still packing or in flight. The kernels are the library's
// own sequential mixes (cfa_mix_seq_f32 / cfa_mix_seq_div_f32) on the chunk's slices, so results
// are bit-identical to the single-shot mix. One call, no Python between chunks.
//
// Staging is chunk-major: chunk c holds the n + 1 slices [a_c, b_c) of every model back to back,
// each padded to a multiple of 4 elements so every slice starts 16-byte aligned.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cfa_copypool.h"
#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char* msg);

namespace {

int hfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

using cfa::Copy;

// The process-wide copy pool (cfa_copypool.h: one atomic (generation, helpers) word per run,
// bounded wait). Never destroyed: its workers may outlive static teardown.
cfa::CopyPool& copy_pool() {
  static cfa::CopyPool* pool = new cfa::CopyPool();
  return *pool;
}

constexpr size_t kPiece = size_t(256) << 10;  // bytes per copy job (load balance across threads)

void add_copies(std::vector<Copy>& jobs, void* dst, const void* src, size_t bytes) {
  for (size_t o = 0; o < bytes; o += kPiece)
    jobs.push_back({static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, std::min(kPiece, bytes - o)});
}

inline size_t pad4(size_t m) { return (m + 3) & ~size_t(3); }

}  // namespace

extern "C" size_t cfa_host_mix_staging_elems(const size_t* layer_elems, int L, int n, size_t chunk_elems) {
  if (!layer_elems || L <= 0 || n < 0) return 0;
  size_t P = 0;
  for (int k = 0; k < L; ++k) P += layer_elems[k];
  const size_t step = pad4(std::max<size_t>(chunk_elems, 4));
  size_t total = 0;
  for (size_t a = 0; a < P; a += step) total += size_t(n + 1) * pad4(std::min(step, P - a));
  return total;
}

extern "C" int cfa_host_mix_f32(float* const* out_layers, const float* const* in_layers,
                                const size_t* layer_elems, int L, int n, const float* alphas,
                                const float* divisors, float* staging, size_t staging_elems,
                                float* out_pinned, size_t chunk_elems, int threads, void* stream) {
  if (L <= 0 || !layer_elems || !in_layers || !out_layers) return hfail(CFA_E_INVALID, "hostmix: null layer tables");
  if (n < 0 || (n > 0 && !alphas)) return hfail(CFA_E_INVALID, "hostmix: bad fan-in / alphas");
  if (!staging || !out_pinned) return hfail(CFA_E_INVALID, "hostmix: null pinned buffers");
  size_t P = 0;
  std::vector<size_t> lo(size_t(L) + 1, 0);
  for (int k = 0; k < L; ++k) {
    for (int m = 0; m <= n; ++m)
      if (layer_elems[k] && !in_layers[size_t(m) * L + k]) return hfail(CFA_E_INVALID, "hostmix: null input layer");
    if (layer_elems[k] && !out_layers[k]) return hfail(CFA_E_INVALID, "hostmix: null output layer");
    P += layer_elems[k];
    lo[size_t(k) + 1] = P;
  }
  if (P == 0) return CFA_OK;
  const size_t need = cfa_host_mix_staging_elems(layer_elems, L, n, chunk_elems);
  if (staging_elems < need)
    return hfail(CFA_E_INVALID, "hostmix: staging of %zu elements, %zu needed", staging_elems, need);
  void *dstage = nullptr, *dout = nullptr;
  if (int rc = cfa_host_device_pointer(staging, &dstage)) return rc;
  if (int rc = cfa_host_device_pointer(out_pinned, &dout)) return rc;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t step = pad4(std::max<size_t>(chunk_elems, 4));
  const int nthreads = std::max(1, std::min(threads, 64));
  cfa::CopyPool& pool = copy_pool();

  struct Chunk {
    size_t a, b, off;
    hipEvent_t ev;
  };
  std::vector<Chunk> chunks;
  for (size_t a = 0, off = 0; a < P; a += step) {
    const size_t b = std::min(P, a + step);
    chunks.push_back({a, b, off, nullptr});
    off += size_t(n + 1) * pad4(b - a);
  }
  // the pieces of layer k that fall in [a, b): global [x, y)
  auto for_pieces = [&](size_t a, size_t b, auto&& fn) {
    for (int k = 0; k < L; ++k) {
      const size_t x = std::max(a, lo[size_t(k)]), y = std::min(b, lo[size_t(k) + 1]);
      if (x < y) fn(k, x, y);
    }
  };
  int rc = CFA_OK;
  size_t launched = 0, unpacked = 0;
  std::vector<Copy> jobs;
  std::vector<const float*> nb(size_t(std::max(n, 1)));
  auto copy_all = [&](const char* what, size_t c) -> int {
    if (pool.run(jobs.data(), jobs.size(), nthreads)) return CFA_OK;
    // run() returns once no helper is inside a copy any more (bounded by 10 minutes)
    if (pool.stragglers())
      return hfail(CFA_E_HIP, "hostmix: host copy pool did not finish the %s of chunk %zu and %d helper(s) are "
                   "still copying: the caller's buffers must not be released", what, c, pool.stragglers());
    return hfail(CFA_E_HIP, "hostmix: host copy pool did not finish the %s of chunk %zu (pool disabled; "
                 "later calls copy on the calling thread)", what, c);
  };
  auto unpack = [&](size_t c) -> int {
    jobs.clear();
    for_pieces(chunks[c].a, chunks[c].b, [&](int k, size_t x, size_t y) {
      add_copies(jobs, out_layers[k] + (x - lo[size_t(k)]), out_pinned + x, (y - x) * sizeof(float));
    });
    return copy_all("unpack", c);
  };
  for (size_t c = 0; c < chunks.size() && rc == CFA_OK; ++c) {
    Chunk& ch = chunks[c];
    const size_t w = pad4(ch.b - ch.a);
    jobs.clear();
    for (int m = 0; m <= n; ++m) {
      float* row = staging + ch.off + size_t(m) * w;
      for_pieces(ch.a, ch.b, [&](int k, size_t x, size_t y) {
        add_copies(jobs, row + (x - ch.a), in_layers[size_t(m) * L + k] + (x - lo[size_t(k)]), (y - x) * sizeof(float));
      });
    }
    if ((rc = copy_all("pack", c)) != CFA_OK) break;
    float* ds = static_cast<float*>(dstage) + ch.off;
    for (int j = 0; j < n; ++j) nb[size_t(j)] = ds + size_t(j + 1) * w;
    float* dst = static_cast<float*>(dout) + ch.a;
    rc = divisors ? cfa_mix_seq_div_f32(dst, ds, nb.data(), alphas, divisors, n, ch.b - ch.a, st)
                  : cfa_mix_seq_f32(dst, ds, nb.data(), alphas, n, ch.b - ch.a, st);
    if (rc) break;
    if (hipEventCreateWithFlags(&ch.ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ch.ev, st) != hipSuccess) {
      rc = hfail(CFA_E_HIP, "hostmix: event record failed");
      break;
    }
    ++launched;
    // unpack whatever earlier chunks have finished while this one is in flight
    while (rc == CFA_OK && unpacked < c && hipEventQuery(chunks[unpacked].ev) == hipSuccess) rc = unpack(unpacked++);
  }
  if (rc == CFA_OK) {
    for (; unpacked < launched; ++unpacked) {
      if (hipEventSynchronize(chunks[unpacked].ev) != hipSuccess) {
        rc = hfail(CFA_E_HIP, "hostmix: chunk %zu failed", unpacked);
        break;
      }
      if ((rc = unpack(unpacked)) != CFA_OK) break;
    }
  }
  if (rc != CFA_OK) (void)hipStreamSynchronize(st);  // drain: no kernel may still read the staging
  for (Chunk& ch : chunks)
    if (ch.ev) (void)hipEventDestroy(ch.ev);
  return rc;
}
