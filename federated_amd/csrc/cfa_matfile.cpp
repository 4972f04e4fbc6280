// cfa_matfile.cpp — native reader and writer of the MATLAB level-5 files the TF1 drivers exchange
// (host ingress / egress formats).
//
// Every TF1 consensus call publishes its model with scipy.io.savemat and reads each neighbour's
// with scipy.io.loadmat (TF1/consensus/cfa.py:108-117, 131-139; cfa_ongraphs.py:214-223, 282-291;
// cfa_ge_2stage.py:537-606). Those files hold a handful of real numeric matrices (weights1,
// biases1, weights2, biases2, epoch, loss_sample, counter_param, grad_*), uncompressed, as
// scipy writes by default. At the reference's model sizes the scipy calls cost more than the
// mixing itself (savemat alone ≈ 0.2 ms per call on the GPU box's host), so the drop-in reads
// and writes these files natively.
//
// Writer: the byte layout scipy's MatFile5Writer produces (128-byte header with 'IM' endian
// mark, one miMATRIX element per variable: array flags, int32 dimensions, miINT8 name, real data
// in column-major order, small-data-element form for sub-elements of at most 4 bytes, every
// element padded to 8 bytes), so scipy.io.loadmat and MATLAB read them unchanged.
// Reader: uncompressed little-endian level-5 files whose variables are real numeric matrices
// (classes double .. uint64), including scipy's and MATLAB's small-data-element forms. Anything
// else (compressed elements, cells, structs, chars, sparse, complex, big-endian) is refused with
// CFA_E_UNSUPPORTED and the caller falls back to scipy. Every read is bounds-checked.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char* msg);

namespace {

int mfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int mfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

enum : uint32_t {
  miINT8 = 1, miUINT8 = 2, miINT16 = 3, miUINT16 = 4, miINT32 = 5, miUINT32 = 6, miSINGLE = 7,
  miDOUBLE = 9, miINT64 = 12, miUINT64 = 13, miMATRIX = 14, miCOMPRESSED = 15
};
enum : uint32_t { mxDOUBLE = 6, mxUINT64 = 15 };

// element size of a numeric mi type (0 = not a numeric data type)
int mi_size(uint32_t t) {
  switch (t) {
    case miINT8: case miUINT8: return 1;
    case miINT16: case miUINT16: return 2;
    case miINT32: case miUINT32: case miSINGLE: return 4;
    case miDOUBLE: case miINT64: case miUINT64: return 8;
    default: return 0;
  }
}

inline uint32_t le32(const unsigned char* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

struct Cursor {
  const unsigned char* p;
  size_t n;
};

// One data element at c (advances c past it, padding included): type, size, payload pointer.
int read_element(Cursor& c, uint32_t* type, uint32_t* size, const unsigned char** data) {
  if (c.n < 8) return mfail(CFA_E_INVALID, "mat: truncated element tag");
  const uint32_t w0 = le32(c.p);
  if (w0 >> 16) {  // small data element: size in the upper half, payload in the next 4 bytes
    *type = w0 & 0xffff;
    *size = w0 >> 16;
    if (*size > 4) return mfail(CFA_E_INVALID, "mat: small element of %u bytes", *size);
    *data = c.p + 4;
    c.p += 8;
    c.n -= 8;
    return CFA_OK;
  }
  *type = w0;
  *size = le32(c.p + 4);
  const size_t padded = (size_t(*size) + 7) & ~size_t(7);
  if (c.n - 8 < size_t(*size)) return mfail(CFA_E_INVALID, "mat: element of %u bytes past the end", *size);
  *data = c.p + 8;
  const size_t step = 8 + (padded <= c.n - 8 ? padded : size_t(*size));  // the last element may be unpadded
  c.p += step;
  c.n -= step;
  return CFA_OK;
}

}  // namespace

struct cfa_mat {
  std::vector<unsigned char> bytes;
  std::string header;
  std::vector<cfa_mat_var_t> vars;
  std::vector<std::string> names;
};

extern "C" int cfa_mat_read(const char* path, cfa_mat_t** out) {
  if (!path || !out) return mfail(CFA_E_INVALID, "mat: null argument");
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return mfail(CFA_E_INVALID, "mat: cannot open %s", path);
  auto* m = new cfa_mat();
  unsigned char buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof(buf), f)) > 0) m->bytes.insert(m->bytes.end(), buf, buf + got);
  fclose(f);
  const std::vector<unsigned char>& b = m->bytes;
  auto refuse = [&](int rc) {
    delete m;
    return rc;
  };
  if (b.size() < 128) return refuse(mfail(CFA_E_INVALID, "mat: %s is shorter than a level-5 header", path));
  if (!(b[126] == 'I' && b[127] == 'M'))
    return refuse(mfail(CFA_E_UNSUPPORTED, "mat: %s is not a little-endian level-5 file", path));
  size_t hl = 116;
  while (hl > 0 && (b[hl - 1] == 0)) --hl;
  m->header.assign(reinterpret_cast<const char*>(b.data()), hl);
  Cursor c{b.data() + 128, b.size() - 128};
  while (c.n > 0) {
    uint32_t type, size;
    const unsigned char* data;
    if (int rc = read_element(c, &type, &size, &data)) return refuse(rc);
    if (type == miCOMPRESSED) return refuse(mfail(CFA_E_UNSUPPORTED, "mat: compressed element"));
    if (type != miMATRIX) return refuse(mfail(CFA_E_UNSUPPORTED, "mat: top-level element of type %u", type));
    Cursor s{data, size};
    uint32_t t, z;
    const unsigned char* d;
    // array flags: class in the low byte; complex 0x800, global 0x400, logical 0x200
    if (int rc = read_element(s, &t, &z, &d)) return refuse(rc);
    if (t != miUINT32 || z < 8) return refuse(mfail(CFA_E_INVALID, "mat: bad array flags"));
    const uint32_t flags = le32(d);
    const uint32_t cls = flags & 0xff;
    if (cls < mxDOUBLE || cls > mxUINT64 || (flags & 0xe00))
      return refuse(mfail(CFA_E_UNSUPPORTED, "mat: class %u / flags 0x%x is not a real numeric matrix", cls, flags));
    cfa_mat_var_t v{};
    v.mat_class = int(cls);
    if (int rc = read_element(s, &t, &z, &d)) return refuse(rc);
    if (t != miINT32 || z % 4 || z / 4 > CFA_MAT_MAX_DIM || z == 0)
      return refuse(mfail(CFA_E_UNSUPPORTED, "mat: bad dimensions element"));
    v.ndim = int(z / 4);
    size_t count = 1;
    for (int k = 0; k < v.ndim; ++k) {
      const int32_t dk = int32_t(le32(d + 4 * k));
      if (dk < 0) return refuse(mfail(CFA_E_INVALID, "mat: negative dimension"));
      v.dims[k] = dk;
      if (dk && count > UINT32_MAX / size_t(dk))  // a data element holds < 4 GiB
        return refuse(mfail(CFA_E_INVALID, "mat: dimensions overflow"));
      count *= size_t(dk);
    }
    if (int rc = read_element(s, &t, &z, &d)) return refuse(rc);
    if (t != miINT8) return refuse(mfail(CFA_E_INVALID, "mat: bad name element"));
    m->names.emplace_back(reinterpret_cast<const char*>(d), z);
    if (int rc = read_element(s, &t, &z, &d)) return refuse(rc);
    const int es = mi_size(t);
    if (!es) return refuse(mfail(CFA_E_UNSUPPORTED, "mat: data of type %u", t));
    if (size_t(z) != count * size_t(es))
      return refuse(mfail(CFA_E_INVALID, "mat: %u data bytes for %zu elements of %d bytes", z, count, es));
    v.mi_type = int(t);
    v.data = d;
    v.nbytes = z;
    m->vars.push_back(v);
  }
  for (size_t i = 0; i < m->vars.size(); ++i) m->vars[i].name = m->names[i].c_str();
  *out = m;
  return CFA_OK;
}

extern "C" void cfa_mat_free(cfa_mat_t* m) { delete m; }

extern "C" int cfa_mat_num_vars(const cfa_mat_t* m) { return m ? int(m->vars.size()) : 0; }

extern "C" const cfa_mat_var_t* cfa_mat_vars(const cfa_mat_t* m) { return m ? m->vars.data() : nullptr; }

extern "C" const char* cfa_mat_header(const cfa_mat_t* m) { return m ? m->header.c_str() : nullptr; }

namespace {
void put32(std::vector<unsigned char>& o, uint32_t v) {
  unsigned char b[4];
  memcpy(b, &v, 4);
  o.insert(o.end(), b, b + 4);
}
void pad8(std::vector<unsigned char>& o, size_t from) {
  while ((o.size() - from) % 8) o.push_back(0);
}
// write_element of scipy's VarWriter5: small-data form at <= 4 bytes, else tag + data + padding
void element(std::vector<unsigned char>& o, uint32_t type, const void* data, size_t bytes) {
  const auto* p = static_cast<const unsigned char*>(data);
  if (bytes <= 4) {
    put32(o, uint32_t(bytes << 16) | type);
    unsigned char b[4] = {0, 0, 0, 0};
    if (bytes) memcpy(b, p, bytes);
    o.insert(o.end(), b, b + 4);
    return;
  }
  put32(o, type);
  put32(o, uint32_t(bytes));
  const size_t from = o.size();
  o.insert(o.end(), p, p + bytes);
  pad8(o, from);
}
}  // namespace

extern "C" int cfa_mat_write(const char* path, const char* header, int nvars, const cfa_mat_var_t* vars) {
  if (!path || nvars < 0 || (nvars && !vars)) return mfail(CFA_E_INVALID, "mat: null argument");
  std::vector<unsigned char> o(128, 0);
  if (header) memcpy(o.data(), header, strnlen(header, 116));
  o[124] = 0x00;  // version 0x0100, little-endian
  o[125] = 0x01;
  o[126] = 'I';
  o[127] = 'M';
  for (int i = 0; i < nvars; ++i) {
    const cfa_mat_var_t& v = vars[i];
    const int es = mi_size(uint32_t(v.mi_type));
    if (!v.name || !*v.name || strlen(v.name) > 63) return mfail(CFA_E_INVALID, "mat: variable %d name", i);
    if (v.mat_class < int(mxDOUBLE) || v.mat_class > int(mxUINT64) || !es || v.ndim < 2 || v.ndim > CFA_MAT_MAX_DIM)
      return mfail(CFA_E_INVALID, "mat: variable %s: class %d, type %d, %d dims", v.name, v.mat_class, v.mi_type,
                   v.ndim);
    size_t count = 1;
    for (int k = 0; k < v.ndim; ++k) {
      if (v.dims[k] < 0 || v.dims[k] > INT32_MAX) return mfail(CFA_E_INVALID, "mat: variable %s dims", v.name);
      count *= size_t(v.dims[k]);
    }
    if (v.nbytes != count * size_t(es) || (v.nbytes && !v.data))
      return mfail(CFA_E_INVALID, "mat: variable %s: %zu bytes for %zu elements", v.name, size_t(v.nbytes), count);
    put32(o, miMATRIX);
    const size_t size_at = o.size();
    put32(o, 0);  // byte count of the sub-elements, patched below
    const size_t start = o.size();
    const uint32_t flags[2] = {uint32_t(v.mat_class), 0};
    element(o, miUINT32, flags, 8);
    int32_t dims[CFA_MAT_MAX_DIM];
    for (int k = 0; k < v.ndim; ++k) dims[k] = int32_t(v.dims[k]);
    element(o, miINT32, dims, 4 * size_t(v.ndim));
    element(o, miINT8, v.name, strlen(v.name));
    element(o, uint32_t(v.mi_type), v.data, size_t(v.nbytes));
    const uint32_t total = uint32_t(o.size() - start);
    memcpy(o.data() + size_at, &total, 4);
  }
  FILE* f = fopen(path, "wb");
  if (!f) return mfail(CFA_E_INVALID, "mat: cannot create %s", path);
  const size_t put = fwrite(o.data(), 1, o.size(), f);
  const int closed = fclose(f);
  if (put != o.size() || closed != 0) return mfail(CFA_E_INVALID, "mat: short write to %s", path);
  return CFA_OK;
}
