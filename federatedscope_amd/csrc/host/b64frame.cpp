// b64_frame: the framing walk of one gRPC tensor upload, natively.
//
// With the gRPC transport every tensor travels as
// base64(pickle.dumps(tensor)) (federatedscope/core/message.py:8-9,110-124)
// and the reference decodes it with pickle inside the aggregation loop
// (core/auxiliaries/utils.py:95-105).  The device path
// (core/compression/b64wire.py) needs only the FRAMING: dtype, shape,
// stride, storage offset and where the raw storage bytes start in the
// decoded stream, so that the base64 characters covering them can go to
// the GPU undecoded.  This is the same whitelisted opcode walk as
// b64wire._walk (the Python restatement, used when this extension is
// absent), decoding only the 4-character groups the walk reads: ~2 us per
// key instead of ~1 ms in Python.  Nothing is executed: the walker knows
// four globals (torch._utils._rebuild_tensor_v2 / _rebuild_parameter,
// torch.storage._load_from_bytes, collections.OrderedDict) and
// torch.<T>Storage inside the storage record, and applies them symbolically.
//
// b64_frame(text) -> (storage_class, shape, stride, storage_offset,
//                     storage_numel, data_pos, requires_grad, nchars)
// raises ValueError("framing: ...") on anything else.
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Val;
using V = std::shared_ptr<Val>;

struct Val {
  enum Kind {
    NONE, BOOL, INT, BIG, STR, BYTES, TUPLE, LIST, DICT, GLOBAL, STORAGE,
    TENSOR, PERSID, MARKER
  } k = NONE;
  int64_t i = 0;         // INT, BOOL; TENSOR: storage offset
  int64_t a = 0, b = 0;  // BYTES / STORAGE: payload start, length
  std::string s;         // STR; BIG: little-endian bytes; GLOBAL: mod\nname
  std::vector<V> items;  // TUPLE, LIST, PERSID (its tuple), DICT (k, v, ...)
  std::vector<int64_t> size, stride;  // TENSOR
  bool rg = false;                    // TENSOR: requires_grad
};

V mk(Val::Kind k) {
  auto v = std::make_shared<Val>();
  v->k = k;
  return v;
}

struct Fail {
  std::string msg;
};

// ---- base64 text -> decoded bytes, on demand -------------------------------
struct Text {
  const unsigned char *c = nullptr;
  int64_t nchars = 0, size = 0;
  int64_t cached_group = -1;
  unsigned char gb[3] = {0, 0, 0};

  static int sextet(unsigned char ch) {
    if (ch >= 'A' && ch <= 'Z') return ch - 'A';
    if (ch >= 'a' && ch <= 'z') return ch - 'a' + 26;
    if (ch >= '0' && ch <= '9') return ch - '0' + 52;
    if (ch == '+') return 62;
    if (ch == '/') return 63;
    return -1;
  }

  void group(int64_t g) {
    if (g == cached_group) return;
    const unsigned char *p = c + 4 * g;
    uint32_t v = 0;
    const bool last = 4 * g + 4 == nchars;
    for (int j = 0; j < 4; ++j) {
      int x = sextet(p[j]);
      if (x < 0) {
        // '=' pads the last group only (its bytes lie past `size`)
        if (!(last && p[j] == '=' && j >= 2))
          throw Fail{"invalid base64 in the tensor framing"};
        x = 0;
      }
      v = (v << 6) | uint32_t(x);
    }
    gb[0] = (v >> 16) & 255;
    gb[1] = (v >> 8) & 255;
    gb[2] = v & 255;
    cached_group = g;
  }

  void read(int64_t pos, int64_t n, unsigned char *out) {
    if (pos < 0 || n < 0 || pos + n > size)
      throw Fail{"tensor framing truncated"};
    for (int64_t q = 0; q < n; ++q) {
      const int64_t b = pos + q;
      group(b / 3);
      out[q] = gb[b % 3];
    }
  }
};

constexpr int kMaxOps = 4096;
constexpr int64_t kMaxStr = 1 << 16;

enum GlobalSet { OUTER, LEGACY_PLAIN, LEGACY_STORAGE };

const char *const kStorageClasses[] = {
    "FloatStorage", "DoubleStorage", "HalfStorage", "BFloat16Storage",
    "LongStorage", "IntStorage", "ShortStorage", "CharStorage",
    "ByteStorage", "BoolStorage", "ComplexFloatStorage",
    "ComplexDoubleStorage"};
const int kStorageSizes[] = {4, 8, 2, 2, 8, 4, 2, 1, 1, 1, 8, 16};

int storage_index(const std::string &name) {
  for (int j = 0; j < 12; ++j)
    if (name == kStorageClasses[j]) return j;
  return -1;
}

bool is_global(const V &v, const char *mod, const char *name) {
  return v && v->k == Val::GLOBAL &&
         v->s == std::string(mod) + "\n" + name;
}

V reduce(const V &fn, const V &args) {
  if (!fn || fn->k != Val::GLOBAL || !args || args->k != Val::TUPLE)
    throw Fail{"REDUCE of a non-whitelisted callable"};
  const auto &a = args->items;
  if (is_global(fn, "torch.storage", "_load_from_bytes")) {
    if (a.size() != 1 || a[0]->k != Val::BYTES)
      throw Fail{"_load_from_bytes takes one bytes object"};
    auto st = mk(Val::STORAGE);
    st->a = a[0]->a;
    st->b = a[0]->b;
    return st;
  }
  if (is_global(fn, "collections", "OrderedDict")) {
    if (!a.empty()) throw Fail{"backward hooks are not part of an upload"};
    return mk(Val::DICT);
  }
  if (is_global(fn, "torch._utils", "_rebuild_tensor_v2")) {
    if (a.size() != 6 && a.size() != 7)
      throw Fail{"_rebuild_tensor_v2 takes 6 or 7 arguments"};
    if (a.size() == 7 && !(a[6]->k == Val::NONE ||
                           (a[6]->k == Val::DICT && a[6]->items.empty())))
      throw Fail{"tensor metadata is not supported"};
    const V &st = a[0], &off = a[1], &sz = a[2], &sd = a[3], &rg = a[4],
            &hooks = a[5];
    if (st->k != Val::STORAGE || off->k != Val::INT || sz->k != Val::TUPLE ||
        sd->k != Val::TUPLE || rg->k != Val::BOOL || hooks->k != Val::DICT ||
        !hooks->items.empty())
      throw Fail{"malformed _rebuild_tensor_v2 arguments"};
    if (sz->items.size() != sd->items.size())
      throw Fail{"size and stride differ or are not ints"};
    auto t = mk(Val::TENSOR);
    t->a = st->a;
    t->b = st->b;
    t->i = off->i;
    for (size_t j = 0; j < sz->items.size(); ++j) {
      if (sz->items[j]->k != Val::INT || sd->items[j]->k != Val::INT)
        throw Fail{"size and stride differ or are not ints"};
      t->size.push_back(sz->items[j]->i);
      t->stride.push_back(sd->items[j]->i);
    }
    t->rg = rg->i != 0;
    return t;
  }
  if (is_global(fn, "torch._utils", "_rebuild_parameter")) {
    if (a.size() != 3 || a[0]->k != Val::TENSOR || a[1]->k != Val::BOOL ||
        !(a[2]->k == Val::NONE ||
          (a[2]->k == Val::DICT && a[2]->items.empty())))
      throw Fail{"malformed _rebuild_parameter arguments"};
    a[0]->rg = a[1]->i != 0;
    return a[0];
  }
  throw Fail{"REDUCE of a non-whitelisted callable"};
}

// One pickle from pos to its STOP (within end); returns the value, updates
// pos to just past STOP.
V walk(Text &src, int64_t &pos, int64_t end, GlobalSet gs) {
  std::vector<V> stack;
  std::vector<size_t> marks;
  std::vector<V> memo;
  unsigned char buf[16];

  auto rd = [&](int64_t n, unsigned char *out) {
    if (pos + n > end) throw Fail{"pickle runs past its frame"};
    src.read(pos, n, out);
    pos += n;
  };
  auto u8 = [&]() {
    rd(1, buf);
    return int64_t(buf[0]);
  };
  auto le = [&](int n) {  // unsigned little-endian
    rd(n, buf);
    uint64_t v = 0;
    for (int j = n - 1; j >= 0; --j) v = (v << 8) | buf[j];
    return v;
  };
  auto floor_ = [&]() { return marks.empty() ? size_t(0) : marks.back(); };
  auto pop = [&]() {
    if (stack.size() <= floor_()) throw Fail{"pickle stack underflow"};
    V v = stack.back();
    stack.pop_back();
    return v;
  };
  auto pop_mark = [&]() {
    if (marks.empty()) throw Fail{"no MARK on the stack"};
    const size_t m = marks.back();
    marks.pop_back();
    std::vector<V> items(stack.begin() + m, stack.end());
    stack.resize(m);
    return items;
  };
  auto text = [&](int64_t n) {
    if (n > kMaxStr) throw Fail{"string too long in the framing"};
    std::string s(size_t(n), '\0');
    if (n) rd(n, reinterpret_cast<unsigned char *>(&s[0]));
    auto v = mk(Val::STR);
    v->s = std::move(s);
    return v;
  };
  auto line = [&]() {
    std::string s;
    for (;;) {
      rd(1, buf);
      if (buf[0] == '\n') break;
      s.push_back(char(buf[0]));
      if (s.size() > 256) throw Fail{"GLOBAL name too long"};
    }
    return s;
  };
  auto global = [&](const std::string &mod, const std::string &name) {
    bool ok = false;
    if (gs == OUTER)
      ok = (mod == "torch._utils" && (name == "_rebuild_tensor_v2" ||
                                      name == "_rebuild_parameter")) ||
           (mod == "torch.storage" && name == "_load_from_bytes") ||
           (mod == "collections" && name == "OrderedDict");
    else if (gs == LEGACY_STORAGE)
      ok = mod == "torch" && storage_index(name) >= 0;
    if (!ok)
      throw Fail{"refusing global " + mod + "." + name + " in a model update"};
    auto v = mk(Val::GLOBAL);
    v->s = mod + "\n" + name;
    return v;
  };
  auto push_int = [&](int64_t x) {
    auto v = mk(Val::INT);
    v->i = x;
    stack.push_back(v);
  };
  auto memo_put = [&](size_t idx) {
    if (stack.empty()) throw Fail{"PUT of an empty stack"};
    if (idx > 1u << 20) throw Fail{"memo index out of range"};
    if (memo.size() <= idx) memo.resize(idx + 1);
    memo[idx] = stack.back();
  };

  for (int ops = 0; ops < kMaxOps; ++ops) {
    const int op = int(u8());
    switch (op) {
      case 0x80:  // PROTO
        if (u8() > 5) throw Fail{"pickle protocol > 5"};
        break;
      case 0x95:  // FRAME
        rd(8, buf);
        break;
      case 0x2e:  // STOP
        if (stack.size() != 1 || !marks.empty())
          throw Fail{"pickle does not end with one value"};
        return stack[0];
      case 0x28:  // MARK
        marks.push_back(stack.size());
        break;
      case 0x29:  // EMPTY_TUPLE
        stack.push_back(mk(Val::TUPLE));
        break;
      case 0x5d:  // EMPTY_LIST
        stack.push_back(mk(Val::LIST));
        break;
      case 0x7d:  // EMPTY_DICT
        stack.push_back(mk(Val::DICT));
        break;
      case 0x74: {  // TUPLE
        auto t = mk(Val::TUPLE);
        t->items = pop_mark();
        stack.push_back(t);
        break;
      }
      case 0x85: case 0x86: case 0x87: {  // TUPLE1..3
        const size_t k = size_t(op - 0x84);
        if (stack.size() - floor_() < k) throw Fail{"pickle stack underflow"};
        auto t = mk(Val::TUPLE);
        t->items.assign(stack.end() - k, stack.end());
        stack.resize(stack.size() - k);
        stack.push_back(t);
        break;
      }
      case 0x61: {  // APPEND
        V v = pop(), l = pop();
        if (l->k != Val::LIST) throw Fail{"APPEND to a non-list"};
        l->items.push_back(v);
        stack.push_back(l);
        break;
      }
      case 0x65: {  // APPENDS
        auto items = pop_mark();
        V l = pop();
        if (l->k != Val::LIST) throw Fail{"APPENDS to a non-list"};
        l->items.insert(l->items.end(), items.begin(), items.end());
        stack.push_back(l);
        break;
      }
      case 0x73: {  // SETITEM
        V v = pop(), key = pop(), d = pop();
        if (d->k != Val::DICT || key->k != Val::STR)
          throw Fail{"SETITEM on a non-dict"};
        d->items.push_back(key);
        d->items.push_back(v);
        stack.push_back(d);
        break;
      }
      case 0x75: {  // SETITEMS
        auto items = pop_mark();
        V d = pop();
        if (d->k != Val::DICT || items.size() % 2)
          throw Fail{"malformed SETITEMS"};
        for (size_t j = 0; j < items.size(); j += 2)
          if (items[j]->k != Val::STR) throw Fail{"dict key is not a str"};
        d->items.insert(d->items.end(), items.begin(), items.end());
        stack.push_back(d);
        break;
      }
      case 0x4e:  // NONE
        stack.push_back(mk(Val::NONE));
        break;
      case 0x88: case 0x89: {  // NEWTRUE, NEWFALSE
        auto v = mk(Val::BOOL);
        v->i = op == 0x88;
        stack.push_back(v);
        break;
      }
      case 0x4b:  // BININT1
        push_int(u8());
        break;
      case 0x4d:  // BININT2
        push_int(int64_t(le(2)));
        break;
      case 0x4a:  // BININT
        push_int(int64_t(int32_t(uint32_t(le(4)))));
        break;
      case 0x8a: {  // LONG1
        const int64_t n = u8();
        if (n <= 8) {
          uint64_t v = n ? le(int(n)) : 0;
          if (n && n < 8 && (v >> (8 * n - 1)) & 1)  // sign-extend
            v |= ~uint64_t(0) << (8 * n);
          push_int(int64_t(v));
        } else {
          auto v = mk(Val::BIG);
          v->s.resize(size_t(n));
          rd(n, reinterpret_cast<unsigned char *>(&v->s[0]));
          stack.push_back(v);
        }
        break;
      }
      case 0x58:  // BINUNICODE
        stack.push_back(text(int64_t(le(4))));
        break;
      case 0x8c:  // SHORT_BINUNICODE
        stack.push_back(text(u8()));
        break;
      case 0x8d: {  // BINUNICODE8
        const uint64_t n = le(8);
        if (n > uint64_t(kMaxStr)) throw Fail{"string too long"};
        stack.push_back(text(int64_t(n)));
        break;
      }
      case 0x42: case 0x43: case 0x8e: {  // BINBYTES, SHORT_, BINBYTES8
        const uint64_t n = op == 0x42 ? le(4) : op == 0x43 ? uint64_t(u8())
                                                           : le(8);
        if (n > uint64_t(end - pos))
          throw Fail{"bytes object runs past the stream"};
        auto v = mk(Val::BYTES);
        v->a = pos;
        v->b = int64_t(n);
        pos += int64_t(n);
        stack.push_back(v);
        break;
      }
      case 0x63: {  // GLOBAL
        std::string mod = line();
        stack.push_back(global(mod, line()));
        break;
      }
      case 0x93: {  // STACK_GLOBAL
        V name = pop(), mod = pop();
        if (mod->k != Val::STR || name->k != Val::STR)
          throw Fail{"STACK_GLOBAL of non-strings"};
        stack.push_back(global(mod->s, name->s));
        break;
      }
      case 0x94:  // MEMOIZE
        memo_put(memo.size());
        break;
      case 0x71:  // BINPUT
        memo_put(size_t(u8()));
        break;
      case 0x72:  // LONG_BINPUT
        memo_put(size_t(le(4)));
        break;
      case 0x68: case 0x6a: {  // BINGET, LONG_BINGET
        const size_t idx = op == 0x68 ? size_t(u8()) : size_t(le(4));
        if (idx >= memo.size() || !memo[idx])
          throw Fail{"GET of an unset memo slot"};
        stack.push_back(memo[idx]);
        break;
      }
      case 0x52: {  // REDUCE
        V args = pop(), fn = pop();
        stack.push_back(reduce(fn, args));
        break;
      }
      case 0x51: {  // BINPERSID
        auto p = mk(Val::PERSID);
        p->items.push_back(pop());
        stack.push_back(p);
        break;
      }
      default: {
        char m[64];
        std::snprintf(m, sizeof m,
                      "pickle opcode 0x%02x is not part of a tensor upload",
                      op);
        throw Fail{m};
      }
    }
  }
  throw Fail{"tensor framing longer than 4096 opcodes"};
}

// torch/serialization.py MAGIC_NUMBER, little-endian LONG1 payload
const unsigned char kMagic[10] = {0x6c, 0xfc, 0x9c, 0x46, 0xf9,
                                  0x20, 0x6a, 0xa8, 0x50, 0x19};

// A walk's result (b64_frame's tuple, built once the GIL is held).
struct FrameOut {
  int si = -1;
  std::vector<int64_t> size, stride;
  int64_t offset = 0, numel = 0, data_pos = 0, nchars = 0;
  bool rg = false;
};

FrameOut frame(Text &src) {
  int64_t pos = 0;
  V t = walk(src, pos, src.size, OUTER);
  if (pos != src.size) throw Fail{"bytes after the pickle"};
  if (t->k != Val::TENSOR) throw Fail{"the upload is not a tensor"};
  // the legacy torch.save stream inside the storage payload
  int64_t p = t->a;
  const int64_t end = t->a + t->b;
  V magic = walk(src, p, end, LEGACY_PLAIN);
  if (magic->k != Val::BIG || magic->s.size() != 10 ||
      std::memcmp(magic->s.data(), kMagic, 10) != 0)
    throw Fail{"storage payload has no torch magic number"};
  V proto = walk(src, p, end, LEGACY_PLAIN);
  if (proto->k != Val::INT || proto->i != 1001)
    throw Fail{"legacy save protocol is not 1001"};
  V info = walk(src, p, end, LEGACY_PLAIN);
  bool little = false;
  if (info->k == Val::DICT)
    for (size_t j = 0; j + 1 < info->items.size(); j += 2)
      if (info->items[j]->s == "little_endian")
        little = info->items[j + 1]->k == Val::BOOL &&
                 info->items[j + 1]->i == 1;
  if (!little) throw Fail{"storage payload is not little-endian"};
  V rec = walk(src, p, end, LEGACY_STORAGE);
  if (rec->k != Val::PERSID || rec->items.size() != 1 ||
      rec->items[0]->k != Val::TUPLE)
    throw Fail{"storage record is not a persistent id"};
  const auto &pid = rec->items[0]->items;
  if ((pid.size() != 5 && pid.size() != 6) || pid[0]->k != Val::STR ||
      pid[0]->s != "storage")
    throw Fail{"storage record is not a persistent id"};
  if (pid.size() == 6 && pid[5]->k != Val::NONE)
    throw Fail{"storage views are not supported"};
  const V &cls = pid[1], &skey = pid[2], &numel = pid[4];
  int si = -1;
  if (cls->k == Val::GLOBAL && cls->s.rfind("torch\n", 0) == 0)
    si = storage_index(cls->s.substr(6));
  if (si < 0 || skey->k != Val::STR || numel->k != Val::INT || numel->i < 0)
    throw Fail{"malformed storage record"};
  V keys = walk(src, p, end, LEGACY_PLAIN);
  if (keys->k != Val::LIST || keys->items.size() != 1 ||
      keys->items[0]->k != Val::STR || keys->items[0]->s != skey->s)
    throw Fail{"storage key list does not match"};
  unsigned char nb[8];
  if (p + 8 > end) throw Fail{"storage element count missing"};
  src.read(p, 8, nb);
  int64_t n = 0;
  for (int j = 7; j >= 0; --j) n = (n << 8) | nb[j];
  if (n != numel->i) throw Fail{"storage element count mismatch"};
  const int es = kStorageSizes[si];
  if (n > (end - p - 8) / es || p + 8 + es * n != end)
    throw Fail{"storage bytes do not fill the payload"};
  // the tensor inside its storage
  if (t->i < 0) throw Fail{"negative offset, size or stride"};
  bool empty = false;
  for (size_t j = 0; j < t->size.size(); ++j) {
    if (t->size[j] < 0 || t->stride[j] < 0)
      throw Fail{"negative offset, size or stride"};
    empty = empty || t->size[j] == 0;
  }
  if (!empty) {
    // overflow-safe: every term is checked against the storage size
    int64_t last = t->i;
    for (size_t j = 0; j < t->size.size(); ++j) {
      const int64_t span = t->size[j] - 1;
      if (span && t->stride[j] > (n - last) / span)
        throw Fail{"tensor reaches past its storage"};
      last += span * t->stride[j];
    }
    if (last >= n) throw Fail{"tensor reaches past its storage"};
  }
  FrameOut o;
  o.si = si;
  o.size = t->size;
  o.stride = t->stride;
  o.offset = t->i;
  o.numel = n;
  o.data_pos = p + 8;
  o.rg = t->rg;
  o.nchars = src.nchars;
  return o;
}

PyObject *to_py(const FrameOut &o) {
  PyObject *shape = PyTuple_New(Py_ssize_t(o.size.size()));
  PyObject *stride = PyTuple_New(Py_ssize_t(o.size.size()));
  if (!shape || !stride) {
    Py_XDECREF(shape);
    Py_XDECREF(stride);
    return nullptr;
  }
  for (size_t j = 0; j < o.size.size(); ++j) {
    PyTuple_SET_ITEM(shape, Py_ssize_t(j), PyLong_FromLongLong(o.size[j]));
    PyTuple_SET_ITEM(stride, Py_ssize_t(j), PyLong_FromLongLong(o.stride[j]));
  }
  return Py_BuildValue("(sNNLLLOL)", kStorageClasses[o.si], shape, stride,
                       (long long)o.offset, (long long)o.numel,
                       (long long)o.data_pos, o.rg ? Py_True : Py_False,
                       (long long)o.nchars);
}

// The characters of a str (compact ASCII, read in place) or bytes-like
// object; false with a Python error set otherwise.
bool text_of(PyObject *obj, Text &src, Py_buffer &view, bool &have_view) {
  have_view = false;
  if (PyUnicode_Check(obj)) {
    if (PyUnicode_READY(obj) != 0) return false;
    if (!PyUnicode_IS_COMPACT_ASCII(obj)) {
      PyErr_SetString(PyExc_ValueError,
                      "framing: invalid base64 in the tensor framing "
                      "(non-ASCII text)");
      return false;
    }
    src.c = static_cast<const unsigned char *>(PyUnicode_DATA(obj));
    src.nchars = PyUnicode_GET_LENGTH(obj);
    return true;
  }
  if (PyObject_GetBuffer(obj, &view, PyBUF_SIMPLE) != 0) return false;
  have_view = true;
  src.c = static_cast<const unsigned char *>(view.buf);
  src.nchars = view.len;
  return true;
}

// The walk of one text, no Python API (runs without the GIL).
FrameOut frame_text(Text &src) {
  if (src.nchars == 0 || src.nchars % 4)
    throw Fail{"base64 text is not a whole number of 4-character groups"};
  int pad = 0;
  if (src.c[src.nchars - 1] == '=') ++pad;
  if (src.c[src.nchars - 2] == '=') ++pad;
  src.size = 3 * (src.nchars / 4) - pad;
  return frame(src);
}

}  // namespace

PyObject *b64_frame(PyObject *, PyObject *args) {
  PyObject *obj;
  if (!PyArg_ParseTuple(args, "O", &obj)) return nullptr;
  Text src;
  Py_buffer view{};
  bool have_view = false;
  if (!text_of(obj, src, view, have_view)) return nullptr;
  PyObject *res = nullptr;
  try {
    res = to_py(frame_text(src));
  } catch (const Fail &f) {
    PyErr_SetString(PyExc_ValueError, ("framing: " + f.msg).c_str());
    res = nullptr;
  } catch (const std::bad_alloc &) {
    PyErr_NoMemory();
    res = nullptr;
  }
  if (have_view) PyBuffer_Release(&view);
  return res;
}

// b64_frame_many(texts[, threads]) -> [b64_frame(text) or None]: the walks
// of every key of one upload, spread over `threads` threads with the GIL
// released (a many-key model pays one call, not one walk per key in
// series).  An entry is None when that text is not a tensor upload (its
// b64_frame would raise); the caller decodes it on the host.
PyObject *b64_frame_many(PyObject *, PyObject *args) {
  PyObject *seq;
  int threads = 8;
  if (!PyArg_ParseTuple(args, "O|i", &seq, &threads)) return nullptr;
  PyObject *fast = PySequence_Fast(seq, "b64_frame_many takes a sequence");
  if (!fast) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  std::vector<Text> src(static_cast<size_t>(n));
  std::vector<Py_buffer> views(static_cast<size_t>(n));
  std::vector<char> have(static_cast<size_t>(n), 0), ok(static_cast<size_t>(n), 0);
  std::vector<FrameOut> out(static_cast<size_t>(n));
  bool fail = false;
  for (Py_ssize_t i = 0; i < n && !fail; ++i) {
    bool hv = false;
    PyObject *o = PySequence_Fast_GET_ITEM(fast, i);
    if (!text_of(o, src[size_t(i)], views[size_t(i)], hv)) {
      PyErr_Clear();            // not text: left to the host decode
      src[size_t(i)].c = nullptr;
    }
    have[size_t(i)] = hv;
  }
  Py_BEGIN_ALLOW_THREADS
  auto work = [&](int t, int nt) {
    for (Py_ssize_t i = t; i < n; i += nt) {
      if (!src[size_t(i)].c) continue;
      try {
        out[size_t(i)] = frame_text(src[size_t(i)]);
        ok[size_t(i)] = 1;
      } catch (...) {
        ok[size_t(i)] = 0;
      }
    }
  };
  int nt = threads < 1 ? 1 : threads;
  if (Py_ssize_t(nt) > n / 4) nt = int(n / 4) < 1 ? 1 : int(n / 4);
  if (nt == 1) {
    work(0, 1);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work, t, nt);
    for (auto &th : pool) th.join();
  }
  Py_END_ALLOW_THREADS
  for (Py_ssize_t i = 0; i < n; ++i)
    if (have[size_t(i)]) PyBuffer_Release(&views[size_t(i)]);
  PyObject *res = PyList_New(n);
  for (Py_ssize_t i = 0; res && i < n; ++i) {
    PyObject *v = ok[size_t(i)] ? to_py(out[size_t(i)]) : Py_NewRef(Py_None);
    if (!v) {
      Py_CLEAR(res);
      break;
    }
    PyList_SET_ITEM(res, i, v);
  }
  Py_DECREF(fast);
  return res;
}
