// cfa_npy.cpp — native reader of the numpy files the TF2 drivers exchange (host
// ingress formats).
//
// The TF2 consensus and parameter-server modules poll two files per neighbour
// (TF2/MNIST_dataset/consensus/consensus_v3.py:82-141, consensus_v4.py:30-95,
// parameter_server_v2.py:83-164):
//   results/dump_train_variables{k}.npz   np.savez(epoch_count=…, training_end=…): a stored
//                                         (uncompressed) zip of 0-d numeric .npy members;
//   results/dump_train_model{k}.npy       np.save of the Keras weight list as a 1-D object array:
//                                         a .npy header ('|O') followed by a pickle of the
//                                         ndarray, whose elements are the per-layer ndarrays.
// np.load(…, allow_pickle=True) unpickles the model file, building every layer through numpy's
// reconstructors and copying each layer's bytes out of the pickle stream. At the C4 model
// (VGG-1, 4.3 MB) that is ≈0.8 ms per neighbour, and the status archive another ≈0.3 ms, more
// than the whole GPU mix of the call.
//
// Here a file is read once into one buffer and its layers are located in place:
// - .npy with a numeric dtype: the header dict (descr, fortran_order, shape) is parsed and the
//   data is the rest of the file;
// - .npy of dtype object: the pickle stream is walked by a small stack machine that understands
//   exactly the opcodes numpy's ndarray.__reduce__ produces under protocols 3 and 4 (what np.save
//   writes under numpy 1.x and 2.x; both module paths): numpy's _reconstruct, ndarray and dtype as the only callables, tuples,
//   lists, ints, bools, None, strings, bytes, memo references and frames. Each element must be a
//   numeric ndarray, whose raw bytes stay where they are in the buffer. Any other global or
//   opcode is refused, so reading a file executes nothing from it;
// - .npz: the zip's central directory is walked (zip64 fields included), each member must be
//   stored (method 0), its CRC-32 is checked as zipfile does, and it is parsed as a numeric .npy.
// Anything outside that (compressed archives, structured or big-endian dtypes, other pickled
// objects) is refused with CFA_E_UNSUPPORTED and the caller falls back to numpy. Every read is
// bounds-checked, so a file caught half-written fails with CFA_E_INVALID, as np.load raises.
#include <sys/stat.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char* msg);

namespace {

int nfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int nfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

template <typename T>
inline T le(const unsigned char* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

// numeric dtype string ("<f4", "|b1", …) -> item size, or 0 when unsupported
int item_size(const std::string& d) {
  if (d.size() < 3 || (d[0] != '<' && d[0] != '|')) return 0;
  const char kind = d[1];
  if (kind != 'f' && kind != 'i' && kind != 'u' && kind != 'b') return 0;
  int sz = 0;
  for (size_t i = 2; i < d.size(); ++i) {
    if (d[i] < '0' || d[i] > '9') return 0;
    sz = sz * 10 + (d[i] - '0');
    if (sz > 8) return 0;
  }
  if (kind == 'f' && sz != 2 && sz != 4 && sz != 8) return 0;
  if ((kind == 'i' || kind == 'u') && sz != 1 && sz != 2 && sz != 4 && sz != 8) return 0;
  if (kind == 'b' && sz != 1) return 0;
  if (d[0] == '|' && sz != 1) return 0;  // '|' only for single-byte types
  return sz;
}

// the canonical descr numpy writes for this kind/size ("|u1", "<f4", …)
std::string canonical(char kind, int size) {
  std::string s(size == 1 ? "|" : "<");
  s += kind;
  s += std::to_string(size);
  return s;
}

bool set_shape(cfa_npy_array_t* a, const std::vector<int64_t>& shape) {
  if (shape.size() > CFA_NPY_MAX_DIM) return false;
  a->ndim = int(shape.size());
  for (size_t k = 0; k < shape.size(); ++k) a->shape[k] = shape[k];
  return true;
}

// element count with overflow guard (false on overflow or a negative extent)
bool count_of(const std::vector<int64_t>& shape, int itemsize, size_t* bytes) {
  unsigned __int128 n = 1;
  for (int64_t d : shape) {
    if (d < 0) return false;
    n *= uint64_t(d);
    if (n > (uint64_t(1) << 48)) return false;
  }
  *bytes = size_t(n * uint64_t(itemsize));
  return true;
}

// ---- .npy header (format 1.0 / 2.0 / 3.0) ------------------------------------------------------
// "{'descr': '<f4', 'fortran_order': False, 'shape': (3, 4), }" — parsed, not evaluated.
struct Header {
  std::string descr;
  bool fortran = false;
  std::vector<int64_t> shape;
};

int parse_header_dict(const char* s, size_t n, Header* h) {
  const std::string t(s, n);
  auto find_key = [&](const char* key) -> size_t {
    const std::string k = std::string("'") + key + "':";
    const size_t p = t.find(k);
    return p == std::string::npos ? p : p + k.size();
  };
  size_t p = find_key("descr");
  if (p == std::string::npos) return nfail(CFA_E_INVALID, "npy: header without descr");
  while (p < n && t[p] == ' ') ++p;
  if (p >= n || t[p] != '\'') return nfail(CFA_E_UNSUPPORTED, "npy: structured dtype");
  const size_t e = t.find('\'', p + 1);
  if (e == std::string::npos) return nfail(CFA_E_INVALID, "npy: bad descr");
  h->descr = t.substr(p + 1, e - p - 1);
  p = find_key("fortran_order");
  if (p == std::string::npos) return nfail(CFA_E_INVALID, "npy: header without fortran_order");
  while (p < n && t[p] == ' ') ++p;
  if (t.compare(p, 4, "True") == 0) h->fortran = true;
  else if (t.compare(p, 5, "False") == 0) h->fortran = false;
  else return nfail(CFA_E_INVALID, "npy: bad fortran_order");
  p = find_key("shape");
  if (p == std::string::npos) return nfail(CFA_E_INVALID, "npy: header without shape");
  while (p < n && t[p] == ' ') ++p;
  if (p >= n || t[p] != '(') return nfail(CFA_E_INVALID, "npy: bad shape");
  ++p;
  h->shape.clear();
  while (p < n && t[p] != ')') {
    if (t[p] == ' ' || t[p] == ',') {
      ++p;
      continue;
    }
    if (t[p] < '0' || t[p] > '9') return nfail(CFA_E_INVALID, "npy: bad shape");
    int64_t v = 0;
    while (p < n && t[p] >= '0' && t[p] <= '9') {
      v = v * 10 + (t[p] - '0');
      if (v > (int64_t(1) << 48)) return nfail(CFA_E_INVALID, "npy: shape overflow");
      ++p;
    }
    h->shape.push_back(v);
  }
  if (p >= n) return nfail(CFA_E_INVALID, "npy: unterminated shape");
  return CFA_OK;
}

// The header of the .npy at b[0..n): fills h, *data_off
int parse_npy_header(const unsigned char* b, size_t n, Header* h, size_t* data_off) {
  static const unsigned char magic[6] = {0x93, 'N', 'U', 'M', 'P', 'Y'};
  if (n < 10) return nfail(CFA_E_INVALID, "npy: truncated header");
  if (memcmp(b, magic, 6) != 0) return nfail(CFA_E_INVALID, "npy: bad magic");
  const int major = b[6];
  size_t hl, off;
  if (major == 1) {
    hl = le<uint16_t>(b + 8);
    off = 10;
  } else if (major == 2 || major == 3) {
    if (n < 12) return nfail(CFA_E_INVALID, "npy: truncated header");
    hl = le<uint32_t>(b + 8);
    off = 12;
  } else {
    return nfail(CFA_E_UNSUPPORTED, "npy: format version %d", major);
  }
  if (n - off < hl) return nfail(CFA_E_INVALID, "npy: truncated header");
  if (int rc = parse_header_dict(reinterpret_cast<const char*>(b + off), hl, h)) return rc;
  *data_off = off + hl;
  return CFA_OK;
}

// ---- the restricted pickle machine for object arrays ------------------------------------------
enum Kind : uint8_t { NONE, BOOL, INT, STR, BYTES, TUPLE, LIST, GLOBAL, DTYPE, NDARRAY };
enum Global : uint8_t { G_RECONSTRUCT, G_NDARRAY, G_DTYPE };

struct Val {
  Kind k;
  int64_t i = 0;                       // INT / BOOL value, GLOBAL id
  const unsigned char* p = nullptr;    // STR / BYTES
  size_t n = 0;
  std::vector<int> items;              // TUPLE / LIST (value indices)
  // DTYPE: descr; NDARRAY: state
  std::string descr;
  bool built = false;
  std::vector<int64_t> shape;
  bool fortran = false;
  int dtype = -1;                      // NDARRAY: index of its DTYPE value
  int data = -1;                       // NDARRAY: BYTES or LIST value
};

class Unpickler {
 public:
  Unpickler(const unsigned char* p, size_t n) : p_(p), end_(p + n) {}

  // Runs to STOP; *result = index of the returned value.
  int run(int* result) {
    for (;;) {
      if (p_ >= end_) return nfail(CFA_E_INVALID, "npy: pickle truncated");
      const unsigned char op = *p_++;
      int rc = CFA_OK;
      switch (op) {
        case 0x80: rc = need(1); if (!rc) { if (p_[0] < 2 || p_[0] > 5) rc = unsup("protocol"); ++p_; } break;  // PROTO
        case 0x95: rc = need(8); if (!rc) p_ += 8; break;                                     // FRAME
        case '.': return finish(result);                                                      // STOP
        case '(': marks_.push_back(stack_.size()); break;                                     // MARK
        case 'N': push(make(NONE)); break;
        case 0x88: push(make_int(BOOL, 1)); break;                                            // NEWTRUE
        case 0x89: push(make_int(BOOL, 0)); break;                                            // NEWFALSE
        case 'K': rc = need(1); if (!rc) { push(make_int(INT, p_[0])); p_ += 1; } break;      // BININT1
        case 'M': rc = need(2); if (!rc) { push(make_int(INT, le<uint16_t>(p_))); p_ += 2; } break;
        case 'J': rc = need(4); if (!rc) { push(make_int(INT, le<int32_t>(p_))); p_ += 4; } break;
        case 0x8a: rc = long1(); break;                                                       // LONG1
        case 0x8c: rc = str_op(1, STR); break;                                                // SHORT_BINUNICODE
        case 'X': rc = str_op(4, STR); break;                                                 // BINUNICODE
        case 0x8d: rc = str_op(8, STR); break;                                                // BINUNICODE8
        case 'C': rc = str_op(1, BYTES); break;                                               // SHORT_BINBYTES
        case 'B': rc = str_op(4, BYTES); break;                                               // BINBYTES
        case 0x8e: rc = str_op(8, BYTES); break;                                              // BINBYTES8
        case 'U': rc = str_op(1, BYTES); break;  // SHORT_BINSTRING (protocol-2 py2 str: numpy's raw data / dtype byte order)
        case 'T': rc = str_op(4, BYTES); break;                                               // BINSTRING
        case ')': push(make(TUPLE)); break;                                                   // EMPTY_TUPLE
        case 't': rc = tuple_mark(); break;                                                   // TUPLE
        case 0x85: rc = tuple_n(1); break;
        case 0x86: rc = tuple_n(2); break;
        case 0x87: rc = tuple_n(3); break;
        case ']': push(make(LIST)); break;                                                    // EMPTY_LIST
        case 'a': rc = append(); break;                                                       // APPEND
        case 'e': rc = appends(); break;                                                      // APPENDS
        case 'c': rc = global_op(); break;                                                    // GLOBAL
        case 0x93: rc = stack_global(); break;                                                // STACK_GLOBAL
        case 'R': rc = reduce(); break;                                                       // REDUCE
        case 'b': rc = build(); break;                                                        // BUILD
        case 0x94: rc = stack_.empty() ? bad("MEMOIZE on empty stack") : (memo_.push_back(stack_.back()), CFA_OK); break;
        case 'q': rc = need(1); if (!rc) { rc = put(p_[0]); p_ += 1; } break;                 // BINPUT
        case 'r': rc = need(4); if (!rc) { rc = put(le<uint32_t>(p_)); p_ += 4; } break;      // LONG_BINPUT
        case 'h': rc = need(1); if (!rc) { rc = get(p_[0]); p_ += 1; } break;                 // BINGET
        case 'j': rc = need(4); if (!rc) { rc = get(le<uint32_t>(p_)); p_ += 4; } break;      // LONG_BINGET
        default: return nfail(CFA_E_UNSUPPORTED, "npy: pickle opcode 0x%02x is outside numpy's array pickles", op);
      }
      if (rc) return rc;
      if (overflow_) return unsup("stream with more than 2^20 objects");
    }
  }

  const Val& val(int i) const { return vals_[size_t(i)]; }

 private:
  int need(size_t k) { return size_t(end_ - p_) < k ? bad("truncated operand") : CFA_OK; }
  static int bad(const char* what) { return nfail(CFA_E_INVALID, "npy: pickle %s", what); }
  static int unsup(const char* what) { return nfail(CFA_E_UNSUPPORTED, "npy: pickle %s not supported", what); }

  int make(Kind k) {
    if (vals_.size() >= kMaxValues) {  // numpy's pickle of an object array makes ~20 values per element
      overflow_ = true;
      return 0;
    }
    vals_.emplace_back();
    vals_.back().k = k;
    return int(vals_.size() - 1);
  }
  int make_int(Kind k, int64_t v) {
    const int i = make(k);
    vals_[size_t(i)].i = v;
    return i;
  }
  void push(int v) { stack_.push_back(v); }
  int pop(int* v) {
    if (stack_.empty() || (!marks_.empty() && stack_.size() <= marks_.back())) return bad("stack underflow");
    *v = stack_.back();
    stack_.pop_back();
    return CFA_OK;
  }

  int long1() {
    if (int rc = need(1)) return rc;
    const size_t n = p_[0];
    ++p_;
    if (n > 8) return unsup("integer wider than 64 bits");
    if (int rc = need(n)) return rc;
    int64_t v = 0;
    for (size_t k = 0; k < n; ++k) v |= int64_t(p_[k]) << (8 * k);
    if (n > 0 && n < 8 && (p_[n - 1] & 0x80)) v -= int64_t(1) << (8 * n);  // sign-extend
    p_ += n;
    push(make_int(INT, v));
    return CFA_OK;
  }

  int str_op(int width, Kind k) {
    if (int rc = need(size_t(width))) return rc;
    uint64_t n = width == 1 ? p_[0] : width == 4 ? le<uint32_t>(p_) : le<uint64_t>(p_);
    p_ += width;
    if (uint64_t(end_ - p_) < n) return bad("string past the end");
    const int i = make(k);
    vals_[size_t(i)].p = p_;
    vals_[size_t(i)].n = size_t(n);
    p_ += n;
    push(i);
    return CFA_OK;
  }

  int tuple_n(size_t n) {
    if (stack_.size() < n + (marks_.empty() ? 0 : marks_.back())) return bad("stack underflow");
    const int t = make(TUPLE);
    vals_[size_t(t)].items.assign(stack_.end() - long(n), stack_.end());
    stack_.resize(stack_.size() - n);
    push(t);
    return CFA_OK;
  }
  int tuple_mark() {
    if (marks_.empty()) return bad("TUPLE without MARK");
    const size_t m = marks_.back();
    marks_.pop_back();
    const int t = make(TUPLE);
    vals_[size_t(t)].items.assign(stack_.begin() + long(m), stack_.end());
    stack_.resize(m);
    push(t);
    return CFA_OK;
  }
  int append() {
    int x;
    if (int rc = pop(&x)) return rc;
    if (stack_.empty() || vals_[size_t(stack_.back())].k != LIST) return bad("APPEND to a non-list");
    vals_[size_t(stack_.back())].items.push_back(x);
    return CFA_OK;
  }
  int appends() {
    if (marks_.empty()) return bad("APPENDS without MARK");
    const size_t m = marks_.back();
    marks_.pop_back();
    if (m == 0 || vals_[size_t(stack_[m - 1])].k != LIST) return bad("APPENDS to a non-list");
    auto& items = vals_[size_t(stack_[m - 1])].items;
    items.insert(items.end(), stack_.begin() + long(m), stack_.end());
    stack_.resize(m);
    return CFA_OK;
  }

  int resolve(const std::string& mod, const std::string& name) {
    int g = -1;
    if ((mod == "numpy.core.multiarray" || mod == "numpy._core.multiarray") && name == "_reconstruct") g = G_RECONSTRUCT;
    else if (mod == "numpy" && name == "ndarray") g = G_NDARRAY;
    else if (mod == "numpy" && name == "dtype") g = G_DTYPE;
    if (g < 0) return nfail(CFA_E_UNSUPPORTED, "npy: pickle global %s.%s is not one of numpy's array reconstructors", mod.c_str(), name.c_str());
    push(make_int(GLOBAL, g));
    return CFA_OK;
  }
  int global_op() {  // GLOBAL "module\nname\n"
    const unsigned char* a = p_;
    const unsigned char* nl1 = static_cast<const unsigned char*>(memchr(a, '\n', size_t(end_ - a)));
    if (!nl1) return bad("GLOBAL truncated");
    const unsigned char* nl2 = static_cast<const unsigned char*>(memchr(nl1 + 1, '\n', size_t(end_ - nl1 - 1)));
    if (!nl2) return bad("GLOBAL truncated");
    p_ = nl2 + 1;
    return resolve(std::string(reinterpret_cast<const char*>(a), size_t(nl1 - a)),
                   std::string(reinterpret_cast<const char*>(nl1 + 1), size_t(nl2 - nl1 - 1)));
  }
  int stack_global() {
    int name, mod;
    if (int rc = pop(&name)) return rc;
    if (int rc = pop(&mod)) return rc;
    const Val& n = vals_[size_t(name)];
    const Val& m = vals_[size_t(mod)];
    if (n.k != STR || m.k != STR) return bad("STACK_GLOBAL of non-strings");
    return resolve(std::string(reinterpret_cast<const char*>(m.p), m.n), std::string(reinterpret_cast<const char*>(n.p), n.n));
  }

  int reduce() {
    int args, fn;
    if (int rc = pop(&args)) return rc;
    if (int rc = pop(&fn)) return rc;
    const Val& f = vals_[size_t(fn)];
    const Val& a = vals_[size_t(args)];
    if (f.k != GLOBAL || a.k != TUPLE) return bad("REDUCE of a non-callable");
    if (f.i == G_RECONSTRUCT) {  // _reconstruct(ndarray, (0,), b'b'): an empty ndarray to BUILD
      if (a.items.size() != 3 || vals_[size_t(a.items[0])].k != GLOBAL || vals_[size_t(a.items[0])].i != G_NDARRAY)
        return unsup("_reconstruct of a non-ndarray");
      push(make(NDARRAY));
      return CFA_OK;
    }
    if (f.i == G_DTYPE) {  // dtype('f4', False, True)
      if (a.items.empty() || vals_[size_t(a.items[0])].k != STR) return bad("dtype without a type string");
      const Val& s = vals_[size_t(a.items[0])];
      const int d = make(DTYPE);
      vals_[size_t(d)].descr.assign(reinterpret_cast<const char*>(s.p), s.n);
      push(d);
      return CFA_OK;
    }
    return unsup("calling ndarray");
  }

  int build() {
    int state, obj;
    if (int rc = pop(&state)) return rc;
    if (int rc = pop(&obj)) return rc;
    const Val& s = vals_[size_t(state)];
    if (s.k != TUPLE) return bad("BUILD with a non-tuple state");
    Val& o = vals_[size_t(obj)];
    if (o.k == DTYPE) {  // (3, '<', None, None, None, -1, -1, flags)
      if (s.items.size() < 2) return bad("dtype state");
      const Val& order = vals_[size_t(s.items[1])];
      if ((order.k != STR && order.k != BYTES) || order.n != 1) return bad("dtype byte order");
      if (s.items.size() >= 3 && vals_[size_t(s.items[2])].k != NONE) return unsup("sub-array dtype");
      if (s.items.size() >= 4 && vals_[size_t(s.items[3])].k != NONE) return unsup("structured dtype");
      const char bo = char(order.p[0]);
      const std::string& t = o.descr;
      if (t == "O8" || t == "O4") {
        o.descr = "|O";
      } else {
        if (t.size() < 2) return unsup("dtype");
        if (bo == '>') return unsup("big-endian dtype");
        int sz = 0;
        for (size_t i = 1; i < t.size(); ++i) {
          if (t[i] < '0' || t[i] > '9') return unsup("dtype");
          sz = sz * 10 + (t[i] - '0');
          if (sz > 8) return unsup("dtype");
        }
        o.descr = canonical(t[0], sz);
        if (!item_size(o.descr)) return unsup("dtype");
      }
      o.built = true;
      push(obj);
      return CFA_OK;
    }
    if (o.k == NDARRAY) {  // (1, shape, dtype, is_fortran, data)
      if (s.items.size() != 5) return bad("ndarray state");
      const Val& shp = vals_[size_t(s.items[1])];
      const Val& dt = vals_[size_t(s.items[2])];
      const Val& fo = vals_[size_t(s.items[3])];
      if (shp.k != TUPLE || dt.k != DTYPE || !dt.built || (fo.k != BOOL && fo.k != INT)) return bad("ndarray state");
      o.shape.clear();
      for (int d : shp.items) {
        if (vals_[size_t(d)].k != INT || vals_[size_t(d)].i < 0) return bad("ndarray shape");
        o.shape.push_back(vals_[size_t(d)].i);
      }
      o.fortran = fo.i != 0;
      o.dtype = s.items[2];
      o.data = s.items[4];
      o.built = true;
      push(obj);
      return CFA_OK;
    }
    return unsup("BUILD of this object");
  }

  int put(uint32_t idx) {
    if (stack_.empty()) return bad("PUT on empty stack");
    if (idx > vals_.size() + 16) return bad("memo index");  // a pickle memoises objects it made
    if (memo_.size() <= idx) memo_.resize(idx + 1, -1);
    memo_[idx] = stack_.back();
    return CFA_OK;
  }
  int get(uint32_t idx) {
    if (idx >= memo_.size() || memo_[idx] < 0) return bad("GET of an unset memo slot");
    push(memo_[idx]);
    return CFA_OK;
  }
  int finish(int* result) {
    if (stack_.size() != 1 || !marks_.empty()) return bad("stack not balanced at STOP");
    *result = stack_.back();
    return CFA_OK;
  }

  static constexpr size_t kMaxValues = size_t(1) << 20;
  const unsigned char* p_;
  const unsigned char* end_;
  bool overflow_ = false;
  std::deque<Val> vals_;  // a deque: references to values stay valid while new ones are made
  std::vector<int> stack_;
  std::vector<size_t> marks_;
  std::vector<int> memo_;
};

uint32_t crc32_of(const unsigned char* p, size_t n) {
  static uint32_t table[256];
  static bool init = [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    return true;
  }();
  (void)init;
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

}  // namespace

struct cfa_npy {
  std::vector<unsigned char> bytes;
  int kind = CFA_NPY_ARRAY;
  std::vector<cfa_npy_array_t> arrays;
  std::vector<std::string> names;
  std::vector<std::string> descrs;
};

namespace {

int read_file(const char* path, std::vector<unsigned char>* out) {
  FILE* f = fopen(path, "rb");
  if (!f) return nfail(CFA_E_INVALID, "npy: cannot open %s", path);
  struct stat st;
  if (fstat(fileno(f), &st) != 0 || st.st_size < 0) {
    fclose(f);
    return nfail(CFA_E_INVALID, "npy: cannot stat %s", path);
  }
  out->resize(size_t(st.st_size));
  const size_t got = out->empty() ? 0 : fread(out->data(), 1, out->size(), f);
  fclose(f);
  if (got != out->size()) return nfail(CFA_E_INVALID, "npy: short read of %s", path);
  return CFA_OK;
}

// one numeric array (a .npy body, an npz member or an object element) appended to m
int add_array(cfa_npy* m, const char* name, const std::string& descr, const std::vector<int64_t>& shape,
              bool fortran, const unsigned char* data, size_t avail, bool exact) {
  const int is = item_size(descr);
  if (!is) return nfail(CFA_E_UNSUPPORTED, "npy: dtype %s", descr.c_str());
  size_t nbytes;
  if (!count_of(shape, is, &nbytes)) return nfail(CFA_E_INVALID, "npy: bad shape");
  if (avail < nbytes || (exact && avail != nbytes))
    return nfail(CFA_E_INVALID, "npy: %zu data bytes for %zu expected", avail, nbytes);
  cfa_npy_array_t a{};
  if (!set_shape(&a, shape)) return nfail(CFA_E_UNSUPPORTED, "npy: more than %d dimensions", CFA_NPY_MAX_DIM);
  a.itemsize = is;
  a.fortran_order = fortran ? 1 : 0;
  a.data = data;
  a.nbytes = nbytes;
  m->arrays.push_back(a);
  m->names.emplace_back(name ? name : "");
  m->descrs.push_back(descr);
  return CFA_OK;
}

int parse_numeric_npy(cfa_npy* m, const char* name, const unsigned char* b, size_t n) {
  Header h;
  size_t off;
  if (int rc = parse_npy_header(b, n, &h, &off)) return rc;
  if (h.descr == "|O") return nfail(CFA_E_UNSUPPORTED, "npy: object member in an archive");
  return add_array(m, name, h.descr, h.shape, h.fortran, b + off, n - off, /*exact=*/true);
}

int parse_object_npy(cfa_npy* m, const Header& h, const unsigned char* b, size_t n) {
  if (h.shape.size() != 1) return nfail(CFA_E_UNSUPPORTED, "npy: object array of %zu dimensions", h.shape.size());
  Unpickler u(b, n);
  int top;
  if (int rc = u.run(&top)) return rc;
  const Val& arr = u.val(top);
  if (arr.k != NDARRAY || !arr.built || u.val(arr.dtype).descr != "|O")
    return nfail(CFA_E_UNSUPPORTED, "npy: pickle is not an object ndarray");
  if (arr.shape != h.shape) return nfail(CFA_E_INVALID, "npy: pickled shape differs from the header");
  const Val& list = u.val(arr.data);
  if (list.k != LIST || int64_t(list.items.size()) != h.shape[0]) return nfail(CFA_E_INVALID, "npy: object array items");
  for (int e : list.items) {
    const Val& el = u.val(e);
    if (el.k != NDARRAY || !el.built) return nfail(CFA_E_UNSUPPORTED, "npy: object element is not an ndarray");
    const Val& dt = u.val(el.dtype);
    const Val& d = u.val(el.data);
    if (dt.descr == "|O" || d.k != BYTES) return nfail(CFA_E_UNSUPPORTED, "npy: nested object array");
    if (int rc = add_array(m, nullptr, dt.descr, el.shape, el.fortran, d.p, d.n, /*exact=*/true)) return rc;
  }
  return CFA_OK;
}

int parse_npz(cfa_npy* m, const unsigned char* b, size_t n) {
  // end of central directory: the last 0x06054b50 within the final 64 KiB + 22 bytes
  if (n < 22) return nfail(CFA_E_INVALID, "npz: truncated archive");
  size_t eocd = SIZE_MAX;
  const size_t lo = n > 65557 ? n - 65557 : 0;
  for (size_t i = n - 22 + 1; i-- > lo;)
    if (le<uint32_t>(b + i) == 0x06054b50u) { eocd = i; break; }
  if (eocd == SIZE_MAX) return nfail(CFA_E_INVALID, "npz: no end-of-central-directory record");
  uint64_t entries = le<uint16_t>(b + eocd + 10);
  uint64_t cd_off = le<uint32_t>(b + eocd + 16);
  if (cd_off == 0xFFFFFFFFu || entries == 0xFFFF) {  // zip64 locator just before the EOCD
    if (eocd < 20 || le<uint32_t>(b + eocd - 20) != 0x07064b50u) return nfail(CFA_E_INVALID, "npz: zip64 locator missing");
    const uint64_t z = le<uint64_t>(b + eocd - 20 + 8);
    if (n < 56 || z > n - 56 || le<uint32_t>(b + z) != 0x06064b50u) return nfail(CFA_E_INVALID, "npz: zip64 record missing");
    entries = le<uint64_t>(b + z + 32);
    cd_off = le<uint64_t>(b + z + 48);
  }
  size_t c = size_t(cd_off);
  if (cd_off > n) return nfail(CFA_E_INVALID, "npz: central directory past the end");
  for (uint64_t e = 0; e < entries; ++e) {
    if (c > n || n - c < 46 || le<uint32_t>(b + c) != 0x02014b50u) return nfail(CFA_E_INVALID, "npz: bad central directory entry");
    const uint16_t flags = le<uint16_t>(b + c + 8);
    const uint16_t method = le<uint16_t>(b + c + 10);
    const uint32_t crc = le<uint32_t>(b + c + 16);
    uint64_t csize = le<uint32_t>(b + c + 20), usize = le<uint32_t>(b + c + 24);
    const size_t nl = le<uint16_t>(b + c + 28), xl = le<uint16_t>(b + c + 30), cl = le<uint16_t>(b + c + 32);
    uint64_t loff = le<uint32_t>(b + c + 42);
    if (n - c - 46 < nl + xl + cl) return nfail(CFA_E_INVALID, "npz: central directory entry past the end");
    std::string name(reinterpret_cast<const char*>(b + c + 46), nl);
    // zip64 extra: the 0xFFFFFFFF fields, in the order usize, csize, offset
    for (size_t x = c + 46 + nl; x + 4 <= c + 46 + nl + xl;) {
      const uint16_t id = le<uint16_t>(b + x), sz = le<uint16_t>(b + x + 2);
      if (x + 4 + sz > c + 46 + nl + xl) return nfail(CFA_E_INVALID, "npz: bad extra field");
      if (id == 1) {
        size_t q = x + 4;
        auto take = [&](uint64_t* v) {
          if (*v != 0xFFFFFFFFu) return true;
          if (q + 8 > x + 4 + sz) return false;
          *v = le<uint64_t>(b + q);
          q += 8;
          return true;
        };
        if (!take(&usize) || !take(&csize) || !take(&loff)) return nfail(CFA_E_INVALID, "npz: bad zip64 extra");
      }
      x += 4 + sz;
    }
    c += 46 + nl + xl + cl;
    if (flags & 1) return nfail(CFA_E_UNSUPPORTED, "npz: encrypted member");
    if (method != 0) return nfail(CFA_E_UNSUPPORTED, "npz: compressed member (np.savez_compressed)");
    if (csize != usize) return nfail(CFA_E_INVALID, "npz: stored member with differing sizes");
    if (loff > n || n - loff < 30 || le<uint32_t>(b + loff) != 0x04034b50u) return nfail(CFA_E_INVALID, "npz: bad local header");
    const uint64_t data = loff + 30 + le<uint16_t>(b + loff + 26) + le<uint16_t>(b + loff + 28);
    if (data > n || n - data < usize) return nfail(CFA_E_INVALID, "npz: member data past the end");
    if (crc32_of(b + data, size_t(usize)) != crc) return nfail(CFA_E_INVALID, "npz: CRC mismatch in %s", name.c_str());
    if (name.size() > 4 && name.compare(name.size() - 4, 4, ".npy") == 0) name.resize(name.size() - 4);
    if (int rc = parse_numeric_npy(m, name.c_str(), b + data, size_t(usize))) return rc;
  }
  return CFA_OK;
}

// The file image b[0..n) (owned by the caller or by m) -> m's arrays
int parse_image(cfa_npy* m, const unsigned char* b, size_t n) {
  if (n >= 4 && le<uint32_t>(b) == 0x04034b50u) {  // PK\3\4: an .npz archive
    m->kind = CFA_NPY_ARCHIVE;
    if (int rc = parse_npz(m, b, n)) return rc;
  } else {
    Header h;
    size_t off;
    if (int rc = parse_npy_header(b, n, &h, &off)) return rc;
    if (h.descr == "|O") {
      m->kind = CFA_NPY_OBJECT;
      if (int rc = parse_object_npy(m, h, b + off, n - off)) return rc;
    } else {
      m->kind = CFA_NPY_ARRAY;
      if (int rc = add_array(m, nullptr, h.descr, h.shape, h.fortran, b + off, n - off, /*exact=*/false)) return rc;
    }
  }
  for (size_t i = 0; i < m->arrays.size(); ++i) {
    m->arrays[i].name = m->kind == CFA_NPY_ARCHIVE ? m->names[i].c_str() : nullptr;
    m->arrays[i].descr = m->descrs[i].c_str();
  }
  return CFA_OK;
}

}  // namespace

extern "C" int cfa_npy_read(const char* path, cfa_npy_t** out) {
  if (!path || !out) return nfail(CFA_E_INVALID, "npy: null argument");
  *out = nullptr;
  auto* m = new cfa_npy();
  int rc = read_file(path, &m->bytes);
  if (!rc) rc = parse_image(m, m->bytes.data(), m->bytes.size());
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return CFA_OK;
}

extern "C" int cfa_npy_parse(const void* image, size_t nbytes, cfa_npy_t** out) {
  if (!out || (!image && nbytes)) return nfail(CFA_E_INVALID, "npy: null argument");
  *out = nullptr;
  auto* m = new cfa_npy();
  static const unsigned char empty = 0;
  if (int rc = parse_image(m, image ? static_cast<const unsigned char*>(image) : &empty, nbytes)) {
    delete m;
    return rc;
  }
  *out = m;
  return CFA_OK;
}

extern "C" void cfa_npy_free(cfa_npy_t* npy) { delete npy; }
extern "C" int cfa_npy_kind(const cfa_npy_t* npy) { return npy ? npy->kind : CFA_E_INVALID; }
extern "C" int cfa_npy_num_arrays(const cfa_npy_t* npy) { return npy ? int(npy->arrays.size()) : 0; }
extern "C" const cfa_npy_array_t* cfa_npy_arrays(const cfa_npy_t* npy) {
  return npy && !npy->arrays.empty() ? npy->arrays.data() : nullptr;
}
