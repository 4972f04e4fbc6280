// cfa_payload.cpp — native codec for the MQTT model payloads of FL_over_MQTT.
//
// The reference ships models between learners and the parameter server as
//   pickle.dumps({'model_layer{k}': w_k.tolist(), 'device': i, 'framecount': f,
//                 'local_epoch': e, 'training_end': b})
// (TF2/FL_over_MQTT/learner_consensus.py:257-268; the PS answers with 'global_model_layer{k}',
// 'global_epoch', 'training_end', PS_server.py:137-149) and decodes them with
//   st = pickle.loads(payload); np.asarray(st['model_layer{k}'])
// (learner_consensus.py:136-144, PS_server.py:90-118), which materialises one Python float per
// parameter before numpy copies them into an fp64 array.
//
// Here the payload bytes are walked once (no Python objects): the structure pass records where
// each list's BINFLOAT runs sit, and the read pass byte-swaps them straight into a caller buffer
// (a pinned staging bucket on the hot path), split over host threads for large tensors. The
// encoder writes the bytes CPython's pickle.dumps writes for the same dict (protocol 2-5,
// framing included), so peers running the reference decode them unchanged.
//
// Only plain containers and scalars are accepted: dict, list, str, int, bool, float, None and
// memo references. Opcodes that construct objects (GLOBAL, STACK_GLOBAL, REDUCE, BUILD, INST,
// OBJ, NEWOBJ, PERSID, EXT) are refused, so decoding a payload executes nothing.
#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cfa_engine.h"

extern "C" void cfa_internal_set_error(const char* msg);

namespace {

int pfail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int pfail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cfa_internal_set_error(buf);
  return code;
}

inline uint64_t load_be64(const unsigned char* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}
inline double be_double(const unsigned char* p) {
  const uint64_t u = load_be64(p);
  double d;
  memcpy(&d, &u, 8);
  return d;
}
template <typename T>
inline T load_le(const unsigned char* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

// ------------------------------------------------------------------------------------------
// Decoded structure.
// ------------------------------------------------------------------------------------------
enum NodeKind : int { K_NONE = 0, K_BOOL, K_INT, K_FLOAT, K_STR, K_LIST, K_DICT };

// A list item: either a run of `count` consecutive BINFLOAT opcodes starting at byte `off`
// (9 bytes each), or one node.
struct Item {
  int64_t off;    // run: byte offset of the first 'G'; node: -1
  int64_t count;  // run: number of floats; node: node id
  bool is_run() const { return off >= 0; }
};

struct Node {
  int kind = K_NONE;
  int64_t ival = 0;  // K_BOOL / K_INT
  double fval = 0;   // K_FLOAT
  int64_t soff = 0, slen = 0;  // K_STR: byte range of the UTF-8 text
  std::vector<Item> items;           // K_LIST
  std::vector<std::pair<int, int>> entries;  // K_DICT: (key node, value node)
};

// Stack entry of the pickle machine: a node, a float run, or a MARK.
struct Slot {
  int64_t off;   // >= 0: float run start; -1: node; -2: mark
  int64_t val;   // run count or node id
};

struct Payload {
  const unsigned char* buf = nullptr;
  size_t len = 0;
  int protocol = 0;
  std::vector<Node> nodes;
  int root = -1;
};

constexpr int kMaxDepth = 64;

int new_node(Payload& P, int kind) {
  P.nodes.emplace_back();
  P.nodes.back().kind = kind;
  return (int)P.nodes.size() - 1;
}

// Turn a slot into a node id (a single float run becomes a K_FLOAT node).
int slot_node(Payload& P, const Slot& s) {
  if (s.off == -1) return (int)s.val;
  const int id = new_node(P, K_FLOAT);
  P.nodes[id].fval = be_double(P.buf + s.off + 1);
  return id;
}

// Expand the slots [b, e) into single values (runs split into one slot per float).
void expand(const std::vector<Slot>& st, size_t b, size_t e, std::vector<Slot>& out) {
  out.clear();
  for (size_t i = b; i < e; ++i) {
    if (st[i].off >= 0)
      for (int64_t k = 0; k < st[i].val; ++k) out.push_back({st[i].off + 9 * k, 1});
    else
      out.push_back(st[i]);
  }
}

const char* opname(unsigned char op) {
  switch (op) {
    case 'c': return "GLOBAL";
    case 0x93: return "STACK_GLOBAL";
    case 'R': return "REDUCE";
    case 'b': return "BUILD";
    case 'i': return "INST";
    case 'o': return "OBJ";
    case 0x81: return "NEWOBJ";
    case 0x92: return "NEWOBJ_EX";
    case 'P': return "PERSID";
    case 'Q': return "BINPERSID";
    case 0x82: case 0x83: case 0x84: return "EXT";
    default: return nullptr;
  }
}

int parse(Payload& P) {
  const unsigned char* b = P.buf;
  const size_t n = P.len;
  std::vector<Slot> st;
  std::vector<size_t> marks;
  std::vector<int> memo;
  std::vector<Slot> tmp;
  size_t i = 0;
  auto need = [&](size_t k) { return i + k <= n; };
  auto pop_mark = [&](size_t& m) -> bool {
    if (marks.empty()) return false;
    m = marks.back();
    marks.pop_back();
    return true;
  };
  auto top_node = [&](int kind, const char* what) -> int {
    if (st.empty() || st.back().off != -1 || P.nodes[st.back().val].kind != kind) {
      pfail(CFA_E_INVALID, "payload: %s without a target container at byte %zu", what, i);
      return -1;
    }
    return (int)st.back().val;
  };
  while (i < n) {
    const size_t at = i;
    const unsigned char op = b[i++];
    switch (op) {
      case 0x80:  // PROTO
        if (!need(1)) goto truncated;
        P.protocol = b[i++];
        if (P.protocol > 5) return pfail(CFA_E_UNSUPPORTED, "payload: pickle protocol %d", P.protocol);
        break;
      case 0x95:  // FRAME: the frame body follows inline
        if (!need(8)) goto truncated;
        if (load_le<uint64_t>(b + i) > n - i - 8) goto truncated;
        i += 8;
        break;
      case '.': {  // STOP
        if (st.size() != 1 || !marks.empty())
          return pfail(CFA_E_INVALID, "payload: malformed stack at STOP (byte %zu)", at);
        P.root = slot_node(P, st[0]);
        return CFA_OK;
      }
      case '}': st.push_back({-1, new_node(P, K_DICT)}); break;
      case ']': st.push_back({-1, new_node(P, K_LIST)}); break;
      case 'N': st.push_back({-1, new_node(P, K_NONE)}); break;
      case 0x88: case 0x89: {  // NEWTRUE / NEWFALSE
        const int id = new_node(P, K_BOOL);
        P.nodes[id].ival = op == 0x88;
        st.push_back({-1, id});
        break;
      }
      case 'K': case 'M': case 'J': {  // BININT1 / BININT2 / BININT
        const size_t k = op == 'K' ? 1 : (op == 'M' ? 2 : 4);
        if (!need(k)) goto truncated;
        const int id = new_node(P, K_INT);
        P.nodes[id].ival = op == 'K' ? b[i] : (op == 'M' ? load_le<uint16_t>(b + i) : load_le<int32_t>(b + i));
        i += k;
        st.push_back({-1, id});
        break;
      }
      case 0x8a: {  // LONG1: little-endian two's complement, up to 8 bytes here
        if (!need(1)) goto truncated;
        const size_t k = b[i++];
        if (!need(k)) goto truncated;
        if (k > 8) return pfail(CFA_E_UNSUPPORTED, "payload: integer wider than 64 bits at byte %zu", at);
        uint64_t u = 0;
        for (size_t q = 0; q < k; ++q) u |= (uint64_t)b[i + q] << (8 * q);
        if (k && k < 8 && (b[i + k - 1] & 0x80)) u |= ~0ULL << (8 * k);  // sign-extend
        const int id = new_node(P, K_INT);
        P.nodes[id].ival = (int64_t)u;
        i += k;
        st.push_back({-1, id});
        break;
      }
      case 'G': {  // BINFLOAT: take the whole run of consecutive BINFLOATs at once
        size_t e = i - 1;
        while (e + 9 <= n && b[e] == 'G') e += 9;
        if (e == at) goto truncated;
        st.push_back({(int64_t)at, (int64_t)((e - at) / 9)});
        i = e;
        break;
      }
      case 0x8c: case 'X': case 0x8d: {  // SHORT_BINUNICODE / BINUNICODE / BINUNICODE8
        const size_t k = op == 0x8c ? 1 : (op == 'X' ? 4 : 8);
        if (!need(k)) goto truncated;
        const uint64_t L = op == 0x8c ? b[i] : (op == 'X' ? load_le<uint32_t>(b + i) : load_le<uint64_t>(b + i));
        i += k;
        if (L > n - i) goto truncated;
        const int id = new_node(P, K_STR);
        P.nodes[id].soff = (int64_t)i;
        P.nodes[id].slen = (int64_t)L;
        i += L;
        st.push_back({-1, id});
        break;
      }
      case '(': marks.push_back(st.size()); break;
      case 0x94: case 'q': case 'r': {  // MEMOIZE / BINPUT / LONG_BINPUT
        if (st.empty()) return pfail(CFA_E_INVALID, "payload: memo of an empty stack at byte %zu", at);
        size_t idx = memo.size();
        if (op != 0x94) {
          const size_t k = op == 'q' ? 1 : 4;
          if (!need(k)) goto truncated;
          idx = op == 'q' ? b[i] : load_le<uint32_t>(b + i);
          i += k;
        }
        Slot& s = st.back();
        if (s.off >= 0 && s.val > 1) {  // only the last float of a run is on top
          Slot last{s.off + 9 * (s.val - 1), 1};
          s.val -= 1;
          st.push_back({-1, slot_node(P, last)});
        } else if (s.off >= 0) {
          st.back() = {-1, slot_node(P, s)};
        }
        if (idx > n) return pfail(CFA_E_INVALID, "payload: memo index %zu out of range", idx);  // bounds memory
        if (memo.size() <= idx) memo.resize(idx + 1, -1);
        memo[idx] = (int)st.back().val;
        break;
      }
      case 'h': case 'j': {  // BINGET / LONG_BINGET
        const size_t k = op == 'h' ? 1 : 4;
        if (!need(k)) goto truncated;
        const size_t idx = op == 'h' ? b[i] : load_le<uint32_t>(b + i);
        i += k;
        if (idx >= memo.size() || memo[idx] < 0)
          return pfail(CFA_E_INVALID, "payload: memo key %zu not found at byte %zu", idx, at);
        st.push_back({-1, memo[idx]});
        break;
      }
      case 'a': {  // APPEND
        if (st.size() < 2) goto underflow;
        const Slot v = st.back();
        st.pop_back();
        const int L = top_node(K_LIST, "APPEND");
        if (L < 0) return CFA_E_INVALID;
        if (v.off >= 0) P.nodes[L].items.push_back({v.off, v.val});
        else P.nodes[L].items.push_back({-1, v.val});
        break;
      }
      case 'e': {  // APPENDS
        size_t m;
        if (!pop_mark(m) || m == 0 || m > st.size()) goto underflow;
        const Slot target = st[m - 1];
        if (target.off != -1 || P.nodes[target.val].kind != K_LIST)
          return pfail(CFA_E_INVALID, "payload: APPENDS without a list at byte %zu", at);
        auto& items = P.nodes[target.val].items;
        for (size_t q = m; q < st.size(); ++q) {
          if (st[q].off >= 0) items.push_back({st[q].off, st[q].val});
          else items.push_back({-1, st[q].val});
        }
        st.resize(m);
        break;
      }
      case 's': case 'u': {  // SETITEM / SETITEMS
        size_t m;
        if (op == 's') {
          if (st.size() < 3) goto underflow;
          m = st.size() - 2;
        } else if (!pop_mark(m) || m == 0 || m > st.size()) {
          goto underflow;
        }
        expand(st, m, st.size(), tmp);
        if (tmp.size() % 2) return pfail(CFA_E_INVALID, "payload: odd SETITEMS at byte %zu", at);
        const Slot target = st[m - 1];
        if (target.off != -1 || P.nodes[target.val].kind != K_DICT)
          return pfail(CFA_E_INVALID, "payload: SETITEM(S) without a dict at byte %zu", at);
        st.resize(m);
        for (size_t q = 0; q < tmp.size(); q += 2) {
          const int k = slot_node(P, tmp[q]), v = slot_node(P, tmp[q + 1]);
          auto& ent = P.nodes[target.val].entries;
          // a repeated key replaces the earlier value (dict semantics)
          bool replaced = false;
          if (P.nodes[k].kind == K_STR) {
            for (auto& kv : ent) {
              const Node& o = P.nodes[kv.first];
              if (o.kind == K_STR && o.slen == P.nodes[k].slen &&
                  !memcmp(b + o.soff, b + P.nodes[k].soff, (size_t)o.slen)) {
                kv.second = v;
                replaced = true;
                break;
              }
            }
          }
          if (!replaced) ent.push_back({k, v});
        }
        break;
      }
      case '0':  // POP
        if (st.empty()) goto underflow;
        if (st.back().off >= 0 && st.back().val > 1) st.back().val -= 1;
        else st.pop_back();
        break;
      default: {
        const char* nm = opname(op);
        if (nm)
          return pfail(CFA_E_INVALID,
                       "payload: opcode %s at byte %zu constructs objects; refused (plain containers only)",
                       nm, at);
        return pfail(CFA_E_UNSUPPORTED, "payload: unsupported pickle opcode 0x%02x at byte %zu", op, at);
      }
    }
  }
truncated:
  return pfail(CFA_E_INVALID, "payload: truncated at byte %zu of %zu", i, n);
underflow:
  return pfail(CFA_E_INVALID, "payload: stack underflow at byte %zu", i);
}

// ------------------------------------------------------------------------------------------
// Array view of a (nested) list: shape and the flat segments in row-major order.
// ------------------------------------------------------------------------------------------
struct Segment {
  int64_t off;    // >= 0: byte offset of a BINFLOAT run; -1: scalar node (val = node id)
  int64_t count;  // elements
  int64_t dst;    // flat destination index
  int64_t node;
};

// Shape of a (nested) list as np.asarray sees it: every list at one depth must have the same
// length and the same kind of items (lists or numbers); `shp` receives this node's shape.
int shape_of(const Payload& P, int id, int depth, std::vector<int64_t>& shp, int& elem_kind) {
  if (depth > kMaxDepth) return pfail(CFA_E_INVALID, "payload: list nesting deeper than %d", kMaxDepth);
  const Node& nd = P.nodes[id];
  shp.clear();
  if (nd.kind != K_LIST) {
    if (nd.kind == K_BOOL || nd.kind == K_INT || nd.kind == K_FLOAT) {
      elem_kind = std::max(elem_kind, nd.kind);
      return CFA_OK;
    }
    return pfail(CFA_E_INVALID, "payload: list holds a non-numeric item");
  }
  int64_t cnt = 0;
  bool has_list = false, has_scalar = false;
  for (const Item& it : nd.items) {
    if (it.is_run()) {
      cnt += it.count;
      has_scalar = true;
      elem_kind = std::max(elem_kind, (int)K_FLOAT);
    } else {
      ++cnt;
      const int k = P.nodes[it.count].kind;
      if (k == K_LIST) {
        has_list = true;
      } else if (k == K_BOOL || k == K_INT || k == K_FLOAT) {
        has_scalar = true;
        elem_kind = std::max(elem_kind, k);
      } else {
        return pfail(CFA_E_INVALID, "payload: list holds a non-numeric item");
      }
    }
  }
  if (has_list && has_scalar) return pfail(CFA_E_INVALID, "payload: ragged nested list");
  std::vector<int64_t> first, cur;
  if (has_list) {
    bool seen = false;
    for (const Item& it : nd.items) {
      const int rc = shape_of(P, (int)it.count, depth + 1, cur, elem_kind);
      if (rc) return rc;
      if (!seen) {
        first = cur;
        seen = true;
      } else if (cur != first) {
        return pfail(CFA_E_INVALID, "payload: ragged nested list at depth %d", depth + 1);
      }
    }
  }
  shp.push_back(cnt);
  shp.insert(shp.end(), first.begin(), first.end());
  return CFA_OK;
}

void segments_of(const Payload& P, int id, std::vector<Segment>& segs, int64_t& pos) {
  const Node& nd = P.nodes[id];
  if (nd.kind != K_LIST) {
    segs.push_back({-1, 1, pos++, id});
    return;
  }
  for (const Item& it : nd.items) {
    if (it.is_run()) {
      segs.push_back({it.off, it.count, pos, -1});
      pos += it.count;
    } else {
      segments_of(P, (int)it.count, segs, pos);
    }
  }
}

const Node* find_key(const Payload& P, const char* key) {
  if (P.root < 0 || P.nodes[P.root].kind != K_DICT) return nullptr;
  const size_t L = strlen(key);
  const Node& d = P.nodes[P.root];
  for (const auto& kv : d.entries) {
    const Node& k = P.nodes[kv.first];
    if (k.kind == K_STR && (size_t)k.slen == L && !memcmp(P.buf + k.soff, key, L)) return &P.nodes[kv.second];
  }
  return nullptr;
}

double scalar_value(const Node& nd) {
  return nd.kind == K_FLOAT ? nd.fval : (double)nd.ival;
}

template <typename T>
void fill_segments(const Payload& P, const std::vector<Segment>& segs, size_t b, size_t e, T* dst) {
  for (size_t s = b; s < e; ++s) {
    const Segment& g = segs[s];
    T* o = dst + g.dst;
    if (g.off >= 0) {
      const unsigned char* p = P.buf + g.off + 1;
      for (int64_t k = 0; k < g.count; ++k, p += 9) o[k] = (T)be_double(p);
    } else {
      o[0] = (T)scalar_value(P.nodes[g.node]);
    }
  }
}

int host_threads(int64_t numel) {
  if (numel < (1 << 20)) return 1;
  unsigned hw = std::thread::hardware_concurrency();
  int t = (int)std::min<int64_t>(numel >> 19, 16);
  if (hw) t = std::min<int>(t, (int)hw);
  return std::max(t, 1);
}

template <typename T>
int read_array(const Payload& P, const char* key, T* dst, int64_t numel) {
  const Node* nd = find_key(P, key);
  if (!nd) return pfail(CFA_E_INVALID, "payload: key '%s' not found", key);
  std::vector<int64_t> shape;
  int ek = K_BOOL;
  int rc = 0;
  const int id = (int)(nd - P.nodes.data());
  if (nd->kind == K_LIST) {
    rc = shape_of(P, id, 0, shape, ek);
    if (rc) return rc;
  } else if (!(nd->kind == K_BOOL || nd->kind == K_INT || nd->kind == K_FLOAT)) {
    return pfail(CFA_E_INVALID, "payload: key '%s' is not numeric", key);
  }
  int64_t total = 1;
  for (int64_t s : shape) total *= s;
  if (total != numel)
    return pfail(CFA_E_INVALID, "payload: key '%s' holds %lld elements, caller expects %lld", key,
                 (long long)total, (long long)numel);
  if (numel == 0) return CFA_OK;
  if (!dst) return pfail(CFA_E_INVALID, "payload: null destination");
  std::vector<Segment> segs;
  int64_t pos = 0;
  segments_of(P, id, segs, pos);
  const int nt = host_threads(numel);
  if (nt == 1 || segs.size() < 2) {
    fill_segments(P, segs, 0, segs.size(), dst);
    return CFA_OK;
  }
  // balance threads by elements: segment ranges with about numel / nt elements each
  std::vector<size_t> cut{0};
  for (int t = 1; t < nt; ++t) {
    const int64_t goal = numel * t / nt;
    size_t s = cut.back();
    while (s < segs.size() && segs[s].dst < goal) ++s;
    cut.push_back(s);
  }
  cut.push_back(segs.size());
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    if (cut[t + 1] > cut[t])
      pool.emplace_back(fill_segments<T>, std::cref(P), std::cref(segs), cut[t], cut[t + 1], dst);
  for (auto& th : pool) th.join();
  return CFA_OK;
}

// ------------------------------------------------------------------------------------------
// Encoder: the byte stream of CPython's pickle.dumps(obj, protocol) for
// {key: ndarray.tolist() | int | bool | float | None}, framing included (protocol >= 4: a frame
// is committed before saving an object once it holds >= 64 KiB; the last frame at STOP; frames
// under 4 bytes carry no header).
// ------------------------------------------------------------------------------------------
class Writer {
 public:
  Writer(unsigned char* dst, size_t cap, int protocol) : dst_(dst), cap_(cap), proto_(protocol) {}
  size_t size() const { return n_; }
  bool dropped_small_frame() const { return dropped_; }
  bool overflow() const { return overflow_; }

  void begin() {
    if (proto_ >= 2) {
      byte(0x80);
      byte((unsigned char)proto_);
    }
    if (proto_ >= 4) open_frame();
  }
  void end() {
    byte('.');
    if (proto_ >= 4) commit_frame(true);
  }
  // called at the start of every object save (pickle.py Pickler.save -> framer.commit_frame)
  void boundary() {
    if (proto_ >= 4 && n_ - fstart_ - 9 >= kFrameTarget) commit_frame(false);
  }
  void byte(unsigned char c) {
    if (n_ < cap_ && dst_) dst_[n_] = c;
    else overflow_ = overflow_ || dst_ != nullptr;
    ++n_;
  }
  void bytes(const void* p, size_t k) {
    if (dst_ && n_ + k <= cap_) memcpy(dst_ + n_, p, k);
    else if (dst_) overflow_ = true;
    n_ += k;
  }
  void memoize() {
    if (proto_ >= 4) {
      byte(0x94);
    } else {  // BINPUT / LONG_BINPUT with an explicit index
      if (memo_ < 256) {
        byte('q');
        byte((unsigned char)memo_);
      } else {
        byte('r');
        const uint32_t v = (uint32_t)memo_;
        bytes(&v, 4);
      }
    }
    ++memo_;
  }
  void save_float(double v) {
    boundary();
    unsigned char rec[9];
    rec[0] = 'G';
    uint64_t u;
    memcpy(&u, &v, 8);
    u = __builtin_bswap64(u);
    memcpy(rec + 1, &u, 8);
    bytes(rec, 9);
  }
  void save_int(int64_t v) {
    boundary();
    if (v >= 0 && v < 256) {
      byte('K');
      byte((unsigned char)v);
    } else if (v >= 0 && v < 65536) {
      byte('M');
      const uint16_t u = (uint16_t)v;
      bytes(&u, 2);
    } else if (v >= INT32_MIN && v <= INT32_MAX) {
      byte('J');
      const int32_t u = (int32_t)v;
      bytes(&u, 4);
    } else {  // LONG1: minimal little-endian two's complement
      unsigned char le[8];
      uint64_t u = (uint64_t)v;
      for (int q = 0; q < 8; ++q) le[q] = (unsigned char)(u >> (8 * q));
      int k = 8;
      while (k > 1 && ((le[k - 1] == 0x00 && !(le[k - 2] & 0x80)) || (le[k - 1] == 0xff && (le[k - 2] & 0x80)))) --k;
      byte(0x8a);
      byte((unsigned char)k);
      bytes(le, (size_t)k);
    }
  }
  void save_bool(bool v) {
    boundary();
    if (proto_ >= 2) {
      byte(v ? 0x88 : 0x89);
    } else {
      bytes(v ? "I01\n" : "I00\n", 4);
    }
  }
  void save_none() {
    boundary();
    byte('N');
  }
  void save_str(const char* s, size_t L) {
    boundary();
    if (L < 256 && proto_ >= 4) {
      byte(0x8c);
      byte((unsigned char)L);
    } else if (L <= 0xffffffffu) {
      byte('X');
      const uint32_t u = (uint32_t)L;
      bytes(&u, 4);
    } else {
      byte(0x8d);
      const uint64_t u = (uint64_t)L;
      bytes(&u, 8);
    }
    bytes(s, L);
    memoize();
  }
  // ndarray.tolist() of a C-contiguous array: nested lists (ndim >= 1) or one float (ndim 0).
  template <typename T>
  void save_array(const T* data, int ndim, const int64_t* shape) {
    if (ndim == 0) {
      save_float((double)data[0]);
      return;
    }
    int64_t inner = 1;
    for (int d = 1; d < ndim; ++d) inner *= shape[d];
    save_list(data, ndim, shape, inner);
  }
  static constexpr size_t kFrameTarget = 64 * 1024;

  // Write the recorded float blocks (BINFLOAT records), split over host threads when large.
  void flush_floats() {
    if (!dst_ || overflow_ || blocks_.empty()) return;
    int64_t total = 0;
    for (const Block& b : blocks_) total += b.count;
    int nt = total < (1 << 20) ? 1 : (int)std::min<int64_t>(total >> 19, 16);
    const unsigned hw = std::thread::hardware_concurrency();
    if (hw) nt = std::min<int>(nt, (int)hw);
    if (nt <= 1) {
      write_blocks(0, blocks_.size());
      return;
    }
    std::vector<size_t> cut{0};
    int64_t acc = 0;
    for (size_t i = 0; i < blocks_.size(); ++i) {
      acc += blocks_[i].count;
      if (acc * nt >= total * (int64_t)cut.size() && cut.size() < (size_t)nt) cut.push_back(i + 1);
    }
    if (cut.back() != blocks_.size()) cut.push_back(blocks_.size());
    std::vector<std::thread> pool;
    for (size_t t = 0; t + 1 < cut.size(); ++t)
      if (cut[t + 1] > cut[t]) pool.emplace_back(&Writer::write_blocks, this, cut[t], cut[t + 1]);
    for (auto& th : pool) th.join();
  }

 private:
  struct Block {
    const void* src;
    bool f32;
    int64_t count;
    size_t off;
  };
  void write_blocks(size_t b, size_t e) {
    for (size_t i = b; i < e; ++i) {
      const Block& bl = blocks_[i];
      unsigned char* o = dst_ + bl.off;
      for (int64_t k = 0; k < bl.count; ++k, o += 9) {
        const double v = bl.f32 ? (double)static_cast<const float*>(bl.src)[k]
                                : static_cast<const double*>(bl.src)[k];
        uint64_t u;
        memcpy(&u, &v, 8);
        u = __builtin_bswap64(u);
        o[0] = 'G';
        memcpy(o + 1, &u, 8);
      }
    }
  }
  // m consecutive floats of one APPENDS batch: the per-object frame check of save_float,
  // evaluated per block (a frame is committed before the float that finds >= 64 KiB in it).
  template <typename T>
  void save_floats(const T* src, int64_t m) {
    while (m > 0) {
      boundary();
      int64_t k = m;
      if (proto_ >= 4) {
        const int64_t cur = (int64_t)(n_ - fstart_ - 9);  // < kFrameTarget after boundary()
        k = std::min<int64_t>(m, ((int64_t)kFrameTarget - cur + 8) / 9);
      }
      if (dst_ && n_ + 9 * (size_t)k <= cap_) blocks_.push_back({src, sizeof(T) == 4, k, n_});
      else if (dst_) overflow_ = true;
      n_ += 9 * (size_t)k;
      src += k;
      m -= k;
    }
  }
  template <typename T>
  void save_list(const T* data, int ndim, const int64_t* shape, int64_t inner) {
    boundary();
    byte(']');
    memoize();
    const int64_t len = shape[0];
    auto item = [&](int64_t k) {
      if (ndim == 1) {
        save_float((double)data[k]);
      } else {
        int64_t in2 = 1;
        for (int d = 2; d < ndim; ++d) in2 *= shape[d];
        save_list(data + k * inner, ndim - 1, shape + 1, in2);
      }
    };
    if (len == 1) {
      item(0);
      byte('a');
    } else if (len > 1) {
      for (int64_t k0 = 0; k0 < len; k0 += 1000) {
        byte('(');
        const int64_t k1 = std::min<int64_t>(len, k0 + 1000);
        if (ndim == 1) {
          save_floats(data + k0, k1 - k0);
        } else {
          for (int64_t k = k0; k < k1; ++k) item(k);
        }
        byte('e');
      }
    }
  }
  void open_frame() {
    fstart_ = n_;
    for (int q = 0; q < 9; ++q) byte(0);
  }
  void commit_frame(bool final_frame) {
    const size_t flen = n_ - fstart_ - 9;
    if (flen >= 4) {
      if (dst_ && fstart_ + 9 <= cap_) {
        dst_[fstart_] = 0x95;
        const uint64_t u = flen;
        memcpy(dst_ + fstart_ + 1, &u, 8);
      }
    } else {  // too small for a header: drop the reserved 9 bytes
      if (dst_ && n_ <= cap_) memmove(dst_ + fstart_, dst_ + fstart_ + 9, flen);
      n_ -= 9;
      dropped_ = true;
    }
    if (!final_frame) open_frame();
  }

  unsigned char* dst_;
  size_t cap_;
  int proto_;
  size_t n_ = 0;
  size_t fstart_ = 0;
  int64_t memo_ = 0;
  bool overflow_ = false;
  bool dropped_ = false;
  std::vector<Block> blocks_;
};

void save_item(Writer& w, const cfa_payload_item_t& it) {
  switch (it.kind) {
    case CFA_PAYLOAD_F32_ARRAY:
      w.save_array(static_cast<const float*>(it.data), it.ndim, it.shape);
      break;
    case CFA_PAYLOAD_F64_ARRAY:
      w.save_array(static_cast<const double*>(it.data), it.ndim, it.shape);
      break;
    case CFA_PAYLOAD_INT: w.save_int(it.ivalue); break;
    case CFA_PAYLOAD_BOOL: w.save_bool(it.ivalue != 0); break;
    case CFA_PAYLOAD_FLOAT: w.save_float(it.fvalue); break;
    default: w.save_none(); break;
  }
}

}  // namespace

extern "C" {

CFA_API int cfa_payload_parse(const void* buf, size_t len, cfa_payload_t** out) {
  if (!out || (!buf && len)) return pfail(CFA_E_INVALID, "payload: null argument");
  *out = nullptr;
  Payload* P = new (std::nothrow) Payload;
  if (!P) return pfail(CFA_E_INVALID, "payload: out of host memory");
  P->buf = static_cast<const unsigned char*>(buf);
  P->len = len;
  int rc;
  try {
    rc = parse(*P);
  } catch (const std::bad_alloc&) {
    rc = pfail(CFA_E_INVALID, "payload: out of host memory while parsing");
  }
  if (rc) {
    delete P;
    return rc;
  }
  if (P->nodes[P->root].kind != K_DICT) {
    delete P;
    return pfail(CFA_E_INVALID, "payload: top-level object is not a dict");
  }
  *out = reinterpret_cast<cfa_payload_t*>(P);
  return CFA_OK;
}

CFA_API void cfa_payload_free(cfa_payload_t* h) { delete reinterpret_cast<Payload*>(h); }

CFA_API int cfa_payload_num_keys(const cfa_payload_t* h) {
  if (!h) return pfail(CFA_E_INVALID, "payload: null handle");
  const Payload& P = *reinterpret_cast<const Payload*>(h);
  return (int)P.nodes[P.root].entries.size();
}

CFA_API int cfa_payload_key(const cfa_payload_t* h, int index, const char** key, size_t* len) {
  if (!h || !key || !len) return pfail(CFA_E_INVALID, "payload: null argument");
  const Payload& P = *reinterpret_cast<const Payload*>(h);
  const auto& ent = P.nodes[P.root].entries;
  if (index < 0 || (size_t)index >= ent.size()) return pfail(CFA_E_INVALID, "payload: key index %d out of range", index);
  const Node& k = P.nodes[ent[index].first];
  if (k.kind != K_STR) return pfail(CFA_E_UNSUPPORTED, "payload: key %d is not a string", index);
  *key = reinterpret_cast<const char*>(P.buf + k.soff);
  *len = (size_t)k.slen;
  return CFA_OK;
}

CFA_API int cfa_payload_info(const cfa_payload_t* h, const char* key, int* kind, int* ndim,
                             int64_t* shape, int64_t* numel) {
  if (!h || !key || !kind || !ndim || !shape || !numel) return pfail(CFA_E_INVALID, "payload: null argument");
  const Payload& P = *reinterpret_cast<const Payload*>(h);
  const Node* nd = find_key(P, key);
  if (!nd) return pfail(CFA_E_INVALID, "payload: key '%s' not found", key);
  *ndim = 0;
  *numel = 1;
  switch (nd->kind) {
    case K_NONE: *kind = CFA_PAYLOAD_NONE; return CFA_OK;
    case K_BOOL: *kind = CFA_PAYLOAD_BOOL; return CFA_OK;
    case K_INT: *kind = CFA_PAYLOAD_INT; return CFA_OK;
    case K_FLOAT: *kind = CFA_PAYLOAD_FLOAT; return CFA_OK;
    case K_STR: *kind = CFA_PAYLOAD_STR; *numel = nd->slen; return CFA_OK;
    case K_DICT: *kind = CFA_PAYLOAD_DICT; *numel = (int64_t)nd->entries.size(); return CFA_OK;
    default: break;
  }
  std::vector<int64_t> shp;
  int ek = K_BOOL;
  const int rc = shape_of(P, (int)(nd - P.nodes.data()), 0, shp, ek);
  if (rc) return rc;
  if (shp.size() > CFA_PAYLOAD_MAX_DIM)
    return pfail(CFA_E_UNSUPPORTED, "payload: key '%s' has %zu dimensions (max %d)", key, shp.size(),
                 CFA_PAYLOAD_MAX_DIM);
  // np.asarray dtype: float64 if any float, else int64 (or bool if every item is a bool);
  // an empty list is float64
  *kind = (ek == K_FLOAT || *numel == 0) ? CFA_PAYLOAD_F64_ARRAY : (ek == K_INT ? CFA_PAYLOAD_I64_ARRAY : CFA_PAYLOAD_BOOL_ARRAY);
  *ndim = (int)shp.size();
  for (size_t d = 0; d < shp.size(); ++d) {
    shape[d] = shp[d];
    *numel *= shp[d];
  }
  if (*numel == 0) *kind = CFA_PAYLOAD_F64_ARRAY;
  return CFA_OK;
}

CFA_API int cfa_payload_scalar(const cfa_payload_t* h, const char* key, int* kind, int64_t* ivalue,
                               double* fvalue) {
  if (!h || !key || !kind || !ivalue || !fvalue) return pfail(CFA_E_INVALID, "payload: null argument");
  const Payload& P = *reinterpret_cast<const Payload*>(h);
  const Node* nd = find_key(P, key);
  if (!nd) return pfail(CFA_E_INVALID, "payload: key '%s' not found", key);
  *ivalue = 0;
  *fvalue = 0;
  switch (nd->kind) {
    case K_NONE: *kind = CFA_PAYLOAD_NONE; return CFA_OK;
    case K_BOOL: *kind = CFA_PAYLOAD_BOOL; *ivalue = nd->ival; *fvalue = (double)nd->ival; return CFA_OK;
    case K_INT: *kind = CFA_PAYLOAD_INT; *ivalue = nd->ival; *fvalue = (double)nd->ival; return CFA_OK;
    case K_FLOAT: *kind = CFA_PAYLOAD_FLOAT; *fvalue = nd->fval; return CFA_OK;
    default: return pfail(CFA_E_INVALID, "payload: key '%s' is not a scalar", key);
  }
}

CFA_API int cfa_payload_read_f64(const cfa_payload_t* h, const char* key, double* dst, int64_t numel) {
  if (!h || !key) return pfail(CFA_E_INVALID, "payload: null argument");
  return read_array(*reinterpret_cast<const Payload*>(h), key, dst, numel);
}

CFA_API int cfa_payload_read_f32(const cfa_payload_t* h, const char* key, float* dst, int64_t numel) {
  if (!h || !key) return pfail(CFA_E_INVALID, "payload: null argument");
  return read_array(*reinterpret_cast<const Payload*>(h), key, dst, numel);
}

CFA_API int cfa_payload_encode(const cfa_payload_item_t* items, int n, int protocol, void* dst,
                               size_t cap, size_t* size) {
  if (!size || n < 0 || (n && !items)) return pfail(CFA_E_INVALID, "payload: null argument");
  if (protocol < 2 || protocol > 5) return pfail(CFA_E_UNSUPPORTED, "payload: protocol %d (2..5 supported)", protocol);
  for (int k = 0; k < n; ++k) {
    const cfa_payload_item_t& it = items[k];
    if (!it.key) return pfail(CFA_E_INVALID, "payload: item %d has no key", k);
    if (it.kind == CFA_PAYLOAD_F32_ARRAY || it.kind == CFA_PAYLOAD_F64_ARRAY) {
      if (it.ndim < 0 || it.ndim > CFA_PAYLOAD_MAX_DIM || (it.ndim && !it.shape))
        return pfail(CFA_E_INVALID, "payload: item '%s' has a bad shape", it.key);
      int64_t numel = 1;
      for (int d = 0; d < it.ndim; ++d) {
        if (it.shape[d] < 0) return pfail(CFA_E_INVALID, "payload: item '%s' has a negative extent", it.key);
        numel *= it.shape[d];
      }
      if (numel && !it.data) return pfail(CFA_E_INVALID, "payload: item '%s' has no data", it.key);
    } else if (it.kind < CFA_PAYLOAD_NONE || it.kind > CFA_PAYLOAD_FLOAT) {
      return pfail(CFA_E_INVALID, "payload: item '%s' has kind %d", it.key, it.kind);
    }
  }
  auto run = [&](unsigned char* out, size_t out_cap, Writer& w) {
    w.begin();
    w.boundary();  // the dict itself
    w.byte('}');
    w.memoize();
    auto pair = [&](int k) {
      w.save_str(items[k].key, strlen(items[k].key));
      save_item(w, items[k]);
    };
    if (n == 1) {
      pair(0);
      w.byte('s');
    } else if (n > 1) {
      for (int k0 = 0; k0 < n; k0 += 1000) {
        w.byte('(');
        for (int k = k0; k < std::min(n, k0 + 1000); ++k) pair(k);
        w.byte('u');
      }
    }
    w.end();
    (void)out;
    (void)out_cap;
  };
  Writer sizer(nullptr, 0, protocol);  // exact length (float blocks are only counted)
  run(nullptr, 0, sizer);
  *size = sizer.size();
  if (!dst) return CFA_OK;
  if (cap < sizer.size())
    return pfail(CFA_E_INVALID, "payload: destination holds %zu bytes, encoding needs %zu", cap, sizer.size());
  if (sizer.dropped_small_frame()) {  // a tiny pickle: the reserved frame header is dropped at
    std::vector<unsigned char> tmp(sizer.size() + 9);  // the end, so write it with headroom
    Writer w(tmp.data(), tmp.size(), protocol);
    run(tmp.data(), tmp.size(), w);
    w.flush_floats();
    memcpy(dst, tmp.data(), w.size());
    return CFA_OK;
  }
  Writer w(static_cast<unsigned char*>(dst), cap, protocol);
  run(static_cast<unsigned char*>(dst), cap, w);
  w.flush_floats();
  if (w.overflow()) return pfail(CFA_E_INVALID, "payload: internal size mismatch");
  return CFA_OK;
}

}  // extern "C"
