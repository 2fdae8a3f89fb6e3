// _fsagg_host: the host half of the row-set boundary (include/fsagg.h
// fsagg_rows), as a CPython extension.
//
// The reference's aggregators walk every client's state_dict key by key in
// Python (clients_avg_aggregator.py:70-91: `for key in avg_model: for i in
// range(len(models)): ... local_model[key]`).  When the uploads are already
// device tensors, the device engine needs exactly one thing from that walk:
// the n x nkeys table of data pointers (and the proof that every tensor is
// a contiguous fp32 tensor of the layout's shape on the right GPU).  Doing
// the walk in Python costs ~1 us per tensor (five attribute reads each);
// here it is one dict lookup and a few inline TensorImpl reads per tensor.
//
// key_table(dicts, keys, shapes, device_index[, offs4])
//   dicts  list of dict (client state_dicts; OrderedDict is a dict)
//   keys   list of str (the layout's fp32 keys, in bucket order)
//   shapes list of tuple[int] (each key's shape, as client 0 holds it)
//   offs4  optional list of int: each key's bucket offset in bytes
// returns (bytes ptrs, int missing, bool aligned16) — ptrs is n*len(keys)
// native int64 data pointers, 0 where a client lacks the key — or None when
// any present value is not a contiguous float32 tensor of that shape on
// cuda:device_index, or an element of dicts is not a dict.  None is not an
// error: the caller then stages the dicts instead.
// With offs4 the table is the device row table itself (include/fsagg.h
// fsagg_rows): segment-major [key][client] virtual bases ptr - offs4[key]
// (0 stays 0), so the caller uploads it as is; the result then carries a
// fourth item, uniform: no key is missing and every client's keys are views
// of one storage at their bucket offsets (one virtual base per client — the
// client's whole bucket is a contiguous range of that storage).
#include <ATen/ATen.h>
#include <Python.h>
#include <torch/csrc/autograd/python_variable.h>

#include <immintrin.h>

#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

// host/b64frame.cpp: the framing walk of one gRPC tensor upload
PyObject *b64_frame(PyObject *, PyObject *args);
PyObject *b64_frame_many(PyObject *, PyObject *args);
// host/krumcert.cpp: the Krum selection certificate
PyObject *gram_select(PyObject *, PyObject *args);

namespace {

PyObject *key_table(PyObject *, PyObject *args) {
  PyObject *dicts, *keys, *shapes, *offs = nullptr;
  int device_index;
  if (!PyArg_ParseTuple(args, "O!O!O!i|O!", &PyList_Type, &dicts,
                        &PyList_Type, &keys, &PyList_Type, &shapes,
                        &device_index, &PyList_Type, &offs))
    return nullptr;
  const Py_ssize_t n = PyList_GET_SIZE(dicts);
  const Py_ssize_t nk = PyList_GET_SIZE(keys);
  if (PyList_GET_SIZE(shapes) != nk ||
      (offs && PyList_GET_SIZE(offs) != nk)) {
    PyErr_SetString(PyExc_ValueError,
                    "keys, shapes and offsets differ in length");
    return nullptr;
  }
  std::vector<int64_t> off4(nk, 0);
  if (offs) {
    for (Py_ssize_t s = 0; s < nk; ++s) {
      off4[s] = PyLong_AsLongLong(PyList_GET_ITEM(offs, s));
      if (off4[s] == -1 && PyErr_Occurred()) return nullptr;
    }
  }
  std::vector<std::vector<int64_t>> shp(nk);
  for (Py_ssize_t s = 0; s < nk; ++s) {
    PyObject *t = PyList_GET_ITEM(shapes, s);
    PyObject *seq = PySequence_Fast(t, "shape must be a sequence");
    if (!seq) return nullptr;
    const Py_ssize_t d = PySequence_Fast_GET_SIZE(seq);
    for (Py_ssize_t j = 0; j < d; ++j) {
      const long long v = PyLong_AsLongLong(PySequence_Fast_GET_ITEM(seq, j));
      if (v == -1 && PyErr_Occurred()) {
        Py_DECREF(seq);
        return nullptr;
      }
      shp[s].push_back(v);
    }
    Py_DECREF(seq);
  }
  std::string buf(size_t(n) * size_t(nk) * sizeof(int64_t), '\0');
  auto *out = reinterpret_cast<int64_t *>(&buf[0]);
  Py_ssize_t missing = 0;
  bool aligned = true;
  // uniform (virtual mode): every client's keys are views of ONE storage at
  // exactly their bucket offsets (one virtual base per client), so the
  // client's bucket is that storage's contiguous range
  bool uniform = offs != nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject *d = PyList_GET_ITEM(dicts, i);
    if (!PyDict_Check(d)) Py_RETURN_NONE;
    int64_t vb0 = 0;
    const void *st0 = nullptr;
    for (Py_ssize_t s = 0; s < nk; ++s) {
      PyObject *v = PyDict_GetItemWithError(d, PyList_GET_ITEM(keys, s));
      // [client][key], or segment-major [key][client] with offsets
      int64_t &slot = offs ? out[s * n + i] : out[i * nk + s];
      if (!v) {
        if (PyErr_Occurred()) return nullptr;
        slot = 0;
        ++missing;
        continue;
      }
      if (!THPVariable_Check(v)) Py_RETURN_NONE;
      // the TensorImpl directly: no Tensor / Storage handles (and their
      // refcount traffic) per key — 16,100 keys at 100 x ResNet-50
      const c10::TensorImpl *t =
          THPVariable_Unpack(v).unsafeGetTensorImpl();
      const c10::Device dv = t->device();
      if (t->dtype() != caffe2::TypeMeta::Make<float>() || !dv.is_cuda() ||
          dv.index() != device_index || !t->is_contiguous())
        Py_RETURN_NONE;
      const auto sz = t->sizes();
      if (sz.size() != shp[s].size()) Py_RETURN_NONE;
      for (size_t j = 0; j < sz.size(); ++j)
        if (sz[j] != shp[s][j]) Py_RETURN_NONE;
      const int64_t numel = t->numel();
      const void *data = t->storage().data();
      const auto p = data == nullptr ? uintptr_t(0)
                                     : reinterpret_cast<uintptr_t>(data) +
                                           uintptr_t(t->storage_offset()) * 4u;
      if (p == 0 && numel > 0) Py_RETURN_NONE;
      aligned = aligned && (p & 15u) == 0;
      slot = p ? int64_t(p) - off4[s] : 0;
      if (uniform) {
        const void *st = data;
        if (numel == 0 || st == nullptr) {
          uniform = false;
        } else if (s == 0) {
          vb0 = slot;
          st0 = st;
        } else if (slot != vb0 || st != st0) {
          uniform = false;
        }
      }
    }
  }
  PyObject *bytes = PyBytes_FromStringAndSize(buf.data(), Py_ssize_t(buf.size()));
  if (!bytes) return nullptr;
  if (offs)
    return Py_BuildValue("(NnOO)", bytes, missing, aligned ? Py_True : Py_False,
                         (uniform && missing == 0 && nk > 0) ? Py_True
                                                             : Py_False);
  return Py_BuildValue("(NnO)", bytes, missing, aligned ? Py_True : Py_False);
}

// device_tensor(ptr, numel, kind, device_index) -> Tensor
// A 1-D tensor over device memory torch does not own (the uncached peer
// buffers fsagg_peer_alloc returns, include/fsagg.h): kind 0 = float32,
// 1 = int32.  No deleter: the caller (core/sharding.PeerAssembly) keeps the
// allocation alive for as long as the tensor is reachable.
PyObject *device_tensor(PyObject *, PyObject *args) {
  unsigned long long ptr;
  long long numel;
  int kind, device_index;
  if (!PyArg_ParseTuple(args, "KLii", &ptr, &numel, &kind, &device_index))
    return nullptr;
  if (ptr == 0 || numel < 0 || kind < 0 || kind > 1 || device_index < 0) {
    PyErr_SetString(PyExc_ValueError, "device_tensor: invalid argument");
    return nullptr;
  }
  auto opts = at::TensorOptions()
                  .dtype(kind == 0 ? at::kFloat : at::kInt)
                  .device(at::Device(at::kCUDA, at::DeviceIndex(device_index)));
  at::Tensor t = at::from_blob(reinterpret_cast<void *>(ptr), {numel}, opts);
  return THPVariable_Wrap(t);
}

// views(flat, spec) -> list[Tensor]
// Views of a flat device bucket in one call: spec is bytes of int64 records
// [ndim, shape[ndim], stride[ndim], offset] (BucketLayout.unpack's per-key
// shape, contiguous strides and bucket offset).  The drop-in's result
// emission made one as_strided call per key from Python (~0.7 us each: 110
// us for the 161 keys of ResNet-50).
PyObject *views(PyObject *, PyObject *args) {
  PyObject *obj;
  Py_buffer spec{};
  if (!PyArg_ParseTuple(args, "Oy*", &obj, &spec)) return nullptr;
  if (!THPVariable_Check(obj)) {
    PyBuffer_Release(&spec);
    PyErr_SetString(PyExc_TypeError, "views: flat must be a tensor");
    return nullptr;
  }
  const at::Tensor &flat = THPVariable_Unpack(obj);
  const auto *r = static_cast<const int64_t *>(spec.buf);
  const size_t nw = size_t(spec.len) / sizeof(int64_t);
  const int64_t base = flat.storage_offset();
  PyObject *out = PyList_New(0);
  size_t i = 0;
  bool ok = out != nullptr;
  while (ok && i < nw) {
    const int64_t nd = r[i];
    if (nd < 0 || i + 2 + 2 * size_t(nd) > nw) {
      PyErr_SetString(PyExc_ValueError, "views: malformed spec");
      ok = false;
      break;
    }
    std::vector<int64_t> shape(r + i + 1, r + i + 1 + nd);
    std::vector<int64_t> stride(r + i + 1 + nd, r + i + 1 + 2 * nd);
    const int64_t off = r[i + 1 + 2 * nd];
    i += 2 + 2 * size_t(nd);
    PyObject *t = THPVariable_Wrap(flat.as_strided(shape, stride, base + off));
    if (!t || PyList_Append(out, t) != 0) ok = false;
    Py_XDECREF(t);
  }
  PyBuffer_Release(&spec);
  if (!ok) {
    Py_XDECREF(out);
    return nullptr;
  }
  return out;
}

// text_copy(text, lo, hi, dst_addr[, threads]) -> None
// Copy characters [lo, hi) of a base64 upload into host memory at dst_addr
// (a pinned staging buffer; core/compression/b64wire.B64Stager).  `text` is
// what the gRPC transport hands the server (federatedscope/core/message.py
// :187-188,236-249): a str — read in place when it is compact ASCII, the
// form CPython keeps base64 text in — or any bytes-like object.  Large
// ranges are copied by several threads with the GIL released.
PyObject *text_copy(PyObject *, PyObject *args) {
  PyObject *obj;
  long long lo, hi;
  unsigned long long dst;
  int threads = 8;
  if (!PyArg_ParseTuple(args, "OLLK|i", &obj, &lo, &hi, &dst, &threads))
    return nullptr;
  const char *src = nullptr;
  Py_ssize_t len = 0;
  Py_buffer view{};
  bool have_view = false;
  if (PyUnicode_Check(obj)) {
    if (PyUnicode_READY(obj) != 0) return nullptr;
    if (!PyUnicode_IS_COMPACT_ASCII(obj)) {
      PyErr_SetString(PyExc_ValueError,
                      "text_copy: base64 text must be ASCII");
      return nullptr;
    }
    src = static_cast<const char *>(PyUnicode_DATA(obj));
    len = PyUnicode_GET_LENGTH(obj);
  } else {
    if (PyObject_GetBuffer(obj, &view, PyBUF_SIMPLE) != 0) return nullptr;
    have_view = true;
    src = static_cast<const char *>(view.buf);
    len = view.len;
  }
  if (lo < 0 || hi < lo || hi > len || dst == 0) {
    if (have_view) PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "text_copy: range out of bounds");
    return nullptr;
  }
  char *out = reinterpret_cast<char *>(dst);
  const size_t n = size_t(hi - lo);
  src += lo;
  Py_BEGIN_ALLOW_THREADS
  const size_t per_min = size_t(4) << 20;  // below 4 MiB a thread is overhead
  int t = threads < 1 ? 1 : threads;
  if (size_t(t) > n / per_min) t = int(n / per_min) < 1 ? 1 : int(n / per_min);
  if (t == 1) {
    std::memcpy(out, src, n);
  } else {
    std::vector<std::thread> pool;
    const size_t step = ((n + t - 1) / t + 4095) & ~size_t(4095);
    for (int i = 0; i < t; ++i) {
      const size_t a = size_t(i) * step;
      if (a >= n) break;
      const size_t b = a + step < n ? a + step : n;
      pool.emplace_back([=] { std::memcpy(out + a, src + a, b - a); });
    }
    for (auto &th : pool) th.join();
  }
  Py_END_ALLOW_THREADS
  if (have_view) PyBuffer_Release(&view);
  Py_RETURN_NONE;
}

// text_copy_many(items, dst_addr[, threads]) -> None: text_copy of every
// (text, lo, hi, off) in `items` to dst_addr + off, the bytes of all items
// split evenly over the threads (one call per upload: a model of many
// small keys copies as fast as one large key).
PyObject *text_copy_many(PyObject *, PyObject *args) {
  PyObject *seq;
  unsigned long long dst;
  int threads = 8;
  if (!PyArg_ParseTuple(args, "OK|i", &seq, &dst, &threads)) return nullptr;
  if (dst == 0) {
    PyErr_SetString(PyExc_ValueError, "text_copy_many: NULL destination");
    return nullptr;
  }
  PyObject *fast = PySequence_Fast(seq, "text_copy_many takes a sequence");
  if (!fast) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  struct Item {
    const char *src;
    char *out;
    size_t n;
  };
  std::vector<Item> items;
  std::vector<Py_buffer> views;
  items.reserve(size_t(n));
  views.reserve(size_t(n));
  bool fail = false;
  for (Py_ssize_t i = 0; i < n && !fail; ++i) {
    PyObject *obj;
    long long lo, hi, off;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(fast, i), "OLLL", &obj,
                          &lo, &hi, &off)) {
      fail = true;
      break;
    }
    const char *src = nullptr;
    Py_ssize_t len = 0;
    if (PyUnicode_Check(obj)) {
      if (PyUnicode_READY(obj) != 0 || !PyUnicode_IS_COMPACT_ASCII(obj)) {
        if (!PyErr_Occurred())
          PyErr_SetString(PyExc_ValueError,
                          "text_copy_many: base64 text must be ASCII");
        fail = true;
        break;
      }
      src = static_cast<const char *>(PyUnicode_DATA(obj));
      len = PyUnicode_GET_LENGTH(obj);
    } else {
      Py_buffer v{};
      if (PyObject_GetBuffer(obj, &v, PyBUF_SIMPLE) != 0) {
        fail = true;
        break;
      }
      views.push_back(v);
      src = static_cast<const char *>(v.buf);
      len = v.len;
    }
    if (lo < 0 || hi < lo || hi > len || off < 0) {
      PyErr_SetString(PyExc_ValueError, "text_copy_many: range out of bounds");
      fail = true;
      break;
    }
    items.push_back({src + lo, reinterpret_cast<char *>(dst) + off,
                     size_t(hi - lo)});
  }
  if (!fail) {
    size_t total = 0;
    for (const auto &it : items) total += it.n;
    Py_BEGIN_ALLOW_THREADS
    // thread t copies bytes [t·step, (t+1)·step) of the items laid end to
    // end
    auto work = [&](size_t a, size_t b) {
      size_t base = 0;
      for (const auto &it : items) {
        const size_t e = base + it.n;
        if (e > a && base < b) {
          const size_t x = a > base ? a - base : 0;
          const size_t y = (b < e ? b : e) - base;
          std::memcpy(it.out + x, it.src + x, y - x);
        }
        base = e;
        if (base >= b) break;
      }
    };
    const size_t per_min = size_t(4) << 20;
    int t = threads < 1 ? 1 : threads;
    if (size_t(t) > total / per_min)
      t = int(total / per_min) < 1 ? 1 : int(total / per_min);
    if (t == 1) {
      work(0, total);
    } else {
      const size_t step = ((total + t - 1) / t + 4095) & ~size_t(4095);
      std::vector<std::thread> pool;
      for (int i = 0; i < t; ++i) {
        const size_t a = size_t(i) * step;
        if (a >= total) break;
        pool.emplace_back(work, a, a + step < total ? a + step : total);
      }
      for (auto &th : pool) th.join();
    }
    Py_END_ALLOW_THREADS
  }
  for (auto &v : views) PyBuffer_Release(&v);
  Py_DECREF(fast);
  if (fail) return nullptr;
  Py_RETURN_NONE;
}

// ---------------------------------------------------------------------------
// host_pack(items, dst_addr[, threads]) -> None
// The host half of the pinned H2D staging of host-resident client updates
// (layout.HostStager): `items` is [(src, nbytes, dst_off)] — src a
// bytes-like object (a CPU fp32 tensor's numpy view) or None for a run of
// zeros (padding, absent keys) — packed into the pinned buffer at dst_addr.
// The bytes of all items are split evenly over a persistent pool of
// threads (no thread start per upload) and written with non-temporal
// stores: the pinned buffer is only read again by the DMA engine, so the
// stores skip the read-for-ownership of each destination line (a third of
// a cached copy's memory traffic).  The GIL is released while the pool
// copies.
namespace {

struct PackItem {
  const char *src;   // nullptr: zeros
  char *out;
  size_t n;
};

__attribute__((target("avx2"))) void nt_copy_avx2(char *d, const char *s,
                                                  size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(d) & 31)) {
    *d++ = s ? *s++ : 0;
    --n;
  }
  const size_t m = n & ~size_t(127);
  if (s) {
    for (size_t i = 0; i < m; i += 128) {
      const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i));
      const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 32));
      const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 64));
      const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + i + 96));
      _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), a);
      _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 32), b);
      _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 64), c);
      _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i + 96), e);
    }
  } else {
    const __m256i z = _mm256_setzero_si256();
    for (size_t i = 0; i < m; i += 32)
      _mm256_stream_si256(reinterpret_cast<__m256i *>(d + i), z);
  }
  _mm_sfence();
  if (s)
    std::memcpy(d + m, s + m, n - m);
  else
    std::memset(d + m, 0, n - m);
}

void plain_copy(char *d, const char *s, size_t n) {
  if (s)
    std::memcpy(d, s, n);
  else
    std::memset(d, 0, n);
}

using CopyFn = void (*)(char *, const char *, size_t);

CopyFn pick_copy() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx2") ? nt_copy_avx2 : plain_copy;
}

// A fixed pool of worker threads, started on first use and kept: each job
// hands every worker one byte range of the concatenated items.
class PackPool {
 public:
  void run(const std::vector<PackItem> &items, size_t total, int threads) {
    std::lock_guard<std::mutex> job(job_mu_);
    if (threads < 1) threads = 1;
    if (threads > kMax) threads = kMax;
    const size_t per_min = size_t(2) << 20;  // below 2 MiB a thread is overhead
    if (size_t(threads) > total / per_min)
      threads = int(total / per_min) < 1 ? 1 : int(total / per_min);
    start(threads - 1);
    const size_t step = ((total + threads - 1) / threads + 4095) & ~size_t(4095);
    {
      std::lock_guard<std::mutex> lk(mu_);
      items_ = &items;
      total_ = total;
      step_ = step;
      active_ = threads - 1;
      pending_ = threads - 1;
      ++gen_;
    }
    cv_.notify_all();
    work(0);                       // the caller takes range 0
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    items_ = nullptr;
  }

 private:
  static constexpr int kMax = 64;
  void start(int want) {
    while (int(workers_.size()) < want) {
      const int id = int(workers_.size()) + 1;
      workers_.emplace_back([this, id] { loop(id); });
      workers_.back().detach();
    }
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      const bool mine = id <= active_;
      lk.unlock();
      if (!mine) continue;
      work(id);
      lk.lock();
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  void work(int part) {
    static const CopyFn copy = pick_copy();
    const size_t a = size_t(part) * step_;
    const size_t b = a + step_ < total_ ? a + step_ : total_;
    if (a >= b) return;
    size_t base = 0;
    for (const auto &it : *items_) {
      const size_t e = base + it.n;
      if (e > a && base < b) {
        const size_t x = a > base ? a - base : 0;
        const size_t y = (b < e ? b : e) - base;
        copy(it.out + x, it.src ? it.src + x : nullptr, y - x);
      }
      base = e;
      if (base >= b) break;
    }
  }
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::vector<PackItem> *items_ = nullptr;
  size_t total_ = 0, step_ = 0;
  int active_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

PackPool *pack_pool() {
  static PackPool *p = new PackPool();   // never destroyed: detached workers
  return p;
}

}  // namespace

PyObject *host_pack(PyObject *, PyObject *args) {
  PyObject *seq;
  unsigned long long dst;
  int threads = 8;
  if (!PyArg_ParseTuple(args, "OK|i", &seq, &dst, &threads)) return nullptr;
  if (dst == 0) {
    PyErr_SetString(PyExc_ValueError, "host_pack: NULL destination");
    return nullptr;
  }
  PyObject *fast = PySequence_Fast(seq, "host_pack takes a sequence");
  if (!fast) return nullptr;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  std::vector<PackItem> items;
  std::vector<Py_buffer> views;
  items.reserve(size_t(n));
  views.reserve(size_t(n));
  bool fail = false;
  for (Py_ssize_t i = 0; i < n && !fail; ++i) {
    PyObject *obj;
    long long nb, off;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(fast, i), "OLL", &obj, &nb,
                          &off)) {
      fail = true;
      break;
    }
    if (nb < 0 || off < 0) {
      PyErr_SetString(PyExc_ValueError, "host_pack: negative size");
      fail = true;
      break;
    }
    const char *src = nullptr;
    if (obj != Py_None) {
      Py_buffer v{};
      if (PyObject_GetBuffer(obj, &v, PyBUF_C_CONTIGUOUS) != 0) {
        fail = true;
        break;
      }
      views.push_back(v);
      if (v.len < nb) {
        PyErr_SetString(PyExc_ValueError, "host_pack: source too short");
        fail = true;
        break;
      }
      src = static_cast<const char *>(v.buf);
    }
    items.push_back({src, reinterpret_cast<char *>(dst) + off, size_t(nb)});
  }
  if (!fail) {
    size_t total = 0;
    for (const auto &it : items) total += it.n;
    Py_BEGIN_ALLOW_THREADS
    pack_pool()->run(items, total, threads);
    Py_END_ALLOW_THREADS
  }
  for (auto &v : views) PyBuffer_Release(&v);
  Py_DECREF(fast);
  if (fail) return nullptr;
  Py_RETURN_NONE;
}

// host_pack_dict(model, spec, zero_runs, dst_addr[, threads]) -> bool
// host_pack with the dict walk in C++: `spec` is [(key, byte offset,
// nbytes, scalar type code, absent_ok)] — each key's CPU tensor, which must
// be contiguous, of that scalar type and exactly nbytes long, goes to
// dst + offset; an absent key (absent_ok) becomes a run of zeros;
// `zero_runs` is [(byte offset, nbytes)] of padding.  Returns False, with
// nothing written, when any present value is not such a tensor or a key
// without absent_ok is missing (the caller then packs in Python).
PyObject *host_pack_dict(PyObject *, PyObject *args) {
  PyObject *model, *spec, *zeros;
  unsigned long long dst;
  int threads = 8;
  if (!PyArg_ParseTuple(args, "OOOK|i", &model, &spec, &zeros, &dst,
                        &threads))
    return nullptr;
  if (!PyDict_Check(model) || dst == 0) Py_RETURN_FALSE;
  PyObject *fs = PySequence_Fast(spec, "host_pack_dict: spec");
  if (!fs) return nullptr;
  PyObject *fz = PySequence_Fast(zeros, "host_pack_dict: zero runs");
  if (!fz) {
    Py_DECREF(fs);
    return nullptr;
  }
  std::vector<PackItem> items;
  const Py_ssize_t ns = PySequence_Fast_GET_SIZE(fs);
  const Py_ssize_t nz = PySequence_Fast_GET_SIZE(fz);
  items.reserve(size_t(ns + nz));
  char *out = reinterpret_cast<char *>(dst);
  bool ok = true, err = false;
  for (Py_ssize_t i = 0; i < ns && ok; ++i) {
    PyObject *key;
    long long off, nb;
    int code, absent_ok;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(fs, i), "OLLii", &key,
                          &off, &nb, &code, &absent_ok)) {
      err = true;
      break;
    }
    PyObject *v = PyDict_GetItemWithError(model, key);   // borrowed
    if (!v) {
      if (PyErr_Occurred()) {
        err = true;
        break;
      }
      if (!absent_ok) {
        ok = false;
        break;
      }
      if (nb) items.push_back({nullptr, out + off, size_t(nb)});
      continue;
    }
    if (!THPVariable_Check(v)) {
      ok = false;
      break;
    }
    const at::Tensor &t = THPVariable_Unpack(v);
    if (!t.device().is_cpu() || int(t.scalar_type()) != code ||
        !t.is_contiguous() || (long long)t.nbytes() != nb) {
      ok = false;
      break;
    }
    if (nb)
      items.push_back({static_cast<const char *>(t.data_ptr()), out + off,
                       size_t(nb)});
  }
  for (Py_ssize_t i = 0; i < nz && ok && !err; ++i) {
    long long off, nb;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(fz, i), "LL", &off, &nb)) {
      err = true;
      break;
    }
    if (nb > 0) items.push_back({nullptr, out + off, size_t(nb)});
  }
  Py_DECREF(fs);
  Py_DECREF(fz);
  if (err) return nullptr;
  if (!ok) Py_RETURN_FALSE;
  size_t total = 0;
  for (const auto &it : items) total += it.n;
  Py_BEGIN_ALLOW_THREADS
  pack_pool()->run(items, total, threads);
  Py_END_ALLOW_THREADS
  Py_RETURN_TRUE;
}

PyMethodDef kMethods[] = {
    {"host_pack_dict", host_pack_dict, METH_VARARGS,
     "host_pack_dict(model, [(key, off, nbytes, dtype_code, absent_ok)], "
     "[(off, nbytes)], dst_addr[, threads]) -> bool"},
    {"host_pack", host_pack, METH_VARARGS,
     "host_pack([(src or None, nbytes, dst_off)], dst_addr[, threads]): "
     "pack host buffers (None: zeros) into pinned memory, non-temporal"},
    {"device_tensor", device_tensor, METH_VARARGS,
     "device_tensor(ptr, numel, kind, device_index) -> Tensor (no ownership)"},
    {"b64_frame", b64_frame, METH_VARARGS,
     "b64_frame(text) -> (storage_class, shape, stride, storage_offset, "
     "storage_numel, data_pos, requires_grad, nchars)"},
    {"b64_frame_many", b64_frame_many, METH_VARARGS,
     "b64_frame_many(texts[, threads]) -> [b64_frame(text) or None]"},
    {"text_copy_many", text_copy_many, METH_VARARGS,
     "text_copy_many([(text, lo, hi, off)], dst_addr[, threads])"},
    {"text_copy", text_copy, METH_VARARGS,
     "text_copy(text, lo, hi, dst_addr[, threads]): copy chars [lo, hi)"},
    {"views", views, METH_VARARGS,
     "views(flat, spec_bytes) -> [Tensor]: as_strided views per record"},
    {"gram_select", gram_select, METH_VARARGS,
     "gram_select(buf, nseg, f, m, ordered) -> None or (scores, order, "
     "ambiguous)"},
    {"key_table", key_table, METH_VARARGS,
     "key_table(dicts, keys, shapes, device_index[, offs4]) -> (bytes, "
     "missing, aligned16) or None"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_fsagg_host",
                       "Host half of libfsagg's row-set boundary.", -1,
                       kMethods};

}  // namespace

PyMODINIT_FUNC PyInit__fsagg_host(void) { return PyModule_Create(&kModule); }
