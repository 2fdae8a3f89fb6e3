// The Krum selection certificate on the host, natively
// (core/aggregators/_engine.ambiguous_clients restated for the common
// case): from the host copy of the Gram path's finish buffer — planes 0-1
// D64 (fp64 [n][n], Σ_key d_key), plane 3 the non-finite flags, plane 4 B
// (fp32, the kernel's bound on |D64 − the exact distances' sum|;
// ops._gram_buf) — the Krum scores (krum_aggregator.py:75-77: the sum of
// each row's n − f − 2 smallest distances), their stable order, and the
// clients whose score intervals keep the selection of the first m from
// being certified.  The Python restatement costs ~30 µs of numpy calls on a
// 50 × 50 matrix; this is a few µs.
//
// gram_select(buf, nseg, f, m, ordered) -> None | (scores, order, amb)
//   buf      a C-contiguous int32 [5][n][n] buffer (numpy array)
//   None     when a pair is flagged (the caller's repair path runs) or
//            n − f − 2 <= 0 (no interval argument applies)
//   scores   bytearray of n fp64 scores, order bytearray of n int64
//   (stable), amb list of int, sorted — empty when the selection is
//   certified.
// Bounds as the Python side forms them: B64 = max(B, Bᵀ) + (nseg + 2)·2^-52
// ·D64 (D64's own fp64 key sum), lo/hi the sums over max(D64 − B64, 0) and
// D64 + B64, scaled by (1 ∓ 1e-12).
#include <Python.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

namespace {

// the sum of a row's k smallest values (their order of addition is the
// selection's: it moves the sum by roundings only, which the intervals'
// 1e-12 slack and the ties the certificate refuses anyway absorb)
double ksum(std::vector<double> &row, int k) {
  std::nth_element(row.begin(), row.begin() + (k - 1), row.end());
  double s = 0.0;
  for (int i = 0; i < k; ++i) s += row[i];
  return s;
}

}  // namespace

PyObject *gram_select(PyObject *, PyObject *args) {
  PyObject *obj;
  int nseg, f, m, ordered;
  if (!PyArg_ParseTuple(args, "Oiiip", &obj, &nseg, &f, &m, &ordered))
    return nullptr;
  Py_buffer view;
  if (PyObject_GetBuffer(obj, &view, PyBUF_C_CONTIGUOUS) != 0) return nullptr;
  const Py_ssize_t words = view.len / 4;
  int n = int(std::lround(std::sqrt(double(words) / 5.0)));
  if (n < 1 || Py_ssize_t(5) * n * n != words) {
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "buffer is not int32 [5][n][n]");
    return nullptr;
  }
  const size_t nn = size_t(n) * n;
  const char *base = static_cast<const char *>(view.buf);
  std::vector<double> D64(nn);
  std::memcpy(D64.data(), base, nn * 8);
  const uint32_t *flag = reinterpret_cast<const uint32_t *>(base + 12 * nn);
  std::vector<float> Bf(nn);
  std::memcpy(Bf.data(), base + 16 * nn, nn * 4);
  PyBuffer_Release(&view);
  const int k = n - f - 2;
  bool flagged = false;
  for (size_t q = 0; q < nn && !flagged; ++q) flagged = flag[q] != 0;
  if (flagged || k <= 0) Py_RETURN_NONE;

  std::vector<double> sc(n), lo(n), hi(n), row(n), rlo(n), rhi(n);
  const double form = (nseg + 2) * std::ldexp(1.0, -52);
  for (int a = 0; a < n; ++a) {
    for (int b = 0; b < n; ++b) {
      const double d = D64[size_t(a) * n + b];
      double bnd = std::max(double(Bf[size_t(a) * n + b]),
                            double(Bf[size_t(b) * n + a]));
      bnd += form * (std::isfinite(d) ? d : 0.0);
      row[b] = d;
      rlo[b] = std::max(d - bnd, 0.0);
      rhi[b] = d + bnd;
    }
    sc[a] = ksum(row, k);
    lo[a] = ksum(rlo, k) * (1 - 1e-12);
    hi[a] = ksum(rhi, k) * (1 + 1e-12);
  }
  std::vector<int> o(n);
  std::iota(o.begin(), o.end(), 0);
  std::stable_sort(o.begin(), o.end(),
                   [&](int x, int y) { return sc[x] < sc[y]; });
  std::vector<char> amb(n, 0);
  if (m > 0) {
    int mm = m;
    bool check = true;
    if (m >= n) {
      if (!ordered) check = false;
      mm = n - 1;
    }
    if (check) {
      // suffix minima of lo in score order
      std::vector<double> suf(n + 1, INFINITY);
      for (int i = n - 1; i >= 0; --i) suf[i] = std::min(suf[i + 1], lo[o[i]]);
      if (!ordered) {
        double top = -INFINITY;
        for (int i = 0; i < mm; ++i) top = std::max(top, hi[o[i]]);
        if (!(top < suf[mm])) {
          for (int i = 0; i < mm; ++i)
            if (hi[o[i]] >= suf[mm]) amb[o[i]] = 1;
          for (int i = mm; i < n; ++i)
            if (lo[o[i]] <= top) amb[o[i]] = 1;
        }
      } else {
        for (int i = 0; i < mm; ++i) {
          if (hi[o[i]] >= suf[i + 1]) {
            amb[o[i]] = 1;
            for (int j = i + 1; j < n; ++j)
              if (lo[o[j]] <= hi[o[i]]) amb[o[j]] = 1;
          }
        }
      }
    }
  }
  std::vector<int64_t> o64(o.begin(), o.end());
  PyObject *ps = PyByteArray_FromStringAndSize(
      reinterpret_cast<const char *>(sc.data()), Py_ssize_t(8) * n);
  PyObject *po = PyByteArray_FromStringAndSize(
      reinterpret_cast<const char *>(o64.data()), Py_ssize_t(8) * n);
  PyObject *pa = PyList_New(0);
  if (!ps || !po || !pa) {
    Py_XDECREF(ps);
    Py_XDECREF(po);
    Py_XDECREF(pa);
    return nullptr;
  }
  for (int i = 0; i < n; ++i) {
    if (amb[i]) {
      PyObject *v = PyLong_FromLong(i);
      PyList_Append(pa, v);
      Py_DECREF(v);
    }
  }
  return Py_BuildValue("(NNN)", ps, po, pa);
}
