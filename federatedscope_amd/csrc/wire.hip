// Wire formats of client uploads, decoded on the device (gfx950):
//
//  * symmetric uniform quantisation (core/compression/utils.py:70-90):
//    the server's dequantisation `value * alpha` (int8/int16 codes times the
//    fp32 0-dim scale, promoted to fp32: one rounding) fused with the scatter
//    of an upload's packed wire bytes into its fp32 client-stack row, so
//    only ~1 B per quantised parameter crosses PCIe;
//  * additive secret sharing (core/secret_sharing/secret_sharing.py:88-98
//    and clients_avg_aggregator.py:79-98): the server sums the clients'
//    fixed-point shares (weight 1.0, numpy float64 semantics), maps the sum
//    back with fixedpoint2float, divides by the total sample size and casts
//    to fp32 — one fused pass instead of np.vectorize per element.
//
// Both are HBM-bound elementwise passes; every arithmetic step is one IEEE
// operation in the reference's order, so the results are bit-exact.
#include <cmath>

#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;
constexpr int kPerThread = 4;
// share rows loaded together (8 measured the same, 16 7 % slower)
constexpr int kSsRows = 8;

struct WireSeg {
  int64_t src;  // byte offset of the segment in the packed upload
  int64_t dst;  // element offset in the fp32 row
  int64_t len;  // elements
  int32_t kind; // FSAGG_WIRE_*
  int32_t scale_idx;  // index into the upload's scale table (-1: none)
};
static_assert(sizeof(WireSeg) == 32, "WireSeg is part of the ABI");

// grid = (ceil(max_len / (kBlock * kPerThread)), nseg): one y-row per
// segment, consecutive threads take consecutive elements.
// Segments are device data the host cannot see at launch time, so each
// block checks its own against the stated extents (src_bytes of packed
// input, out_len of the row) and skips one that does not fit: a malformed
// table writes nothing instead of faulting.
__global__ __launch_bounds__(kBlock) void wire_unpack_kernel(
    const unsigned char *__restrict__ src, const WireSeg *__restrict__ segs,
    const float *__restrict__ scales, int nscale, int64_t src_bytes,
    int64_t out_len, float *__restrict__ out) {
  const WireSeg sg = segs[blockIdx.y];
  const int64_t base = int64_t(blockIdx.x) * kBlock * kPerThread;
  if (base >= sg.len) return;
  const int64_t width = sg.kind == FSAGG_WIRE_I8 ? 1
                        : sg.kind == FSAGG_WIRE_I16 ? 2 : 4;
  if (sg.len < 0 || sg.src < 0 || sg.dst < 0 || sg.src % width ||
      sg.src > src_bytes || sg.len > (src_bytes - sg.src) / width ||
      sg.dst > out_len || sg.len > out_len - sg.dst ||
      (sg.kind != FSAGG_WIRE_F32 && sg.kind != FSAGG_WIRE_I8 &&
       sg.kind != FSAGG_WIRE_I16) ||
      sg.scale_idx >= nscale)
    return;
  const float s = sg.scale_idx >= 0 ? scales[sg.scale_idx] : 1.0f;
#pragma unroll
  for (int e = 0; e < kPerThread; ++e) {
    const int64_t i = base + int64_t(e) * kBlock + threadIdx.x;
    if (i >= sg.len) break;
    float v;
    if (sg.kind == FSAGG_WIRE_I8) {
      v = mul_rn(float(reinterpret_cast<const int8_t *>(src + sg.src)[i]), s);
    } else if (sg.kind == FSAGG_WIRE_I16) {
      v = mul_rn(float(reinterpret_cast<const int16_t *>(src + sg.src)[i]),
                 s);
    } else {  // FSAGG_WIRE_F32: copied as is
      v = reinterpret_cast<const float *>(src + sg.src)[i];
    }
    out[sg.dst + i] = v;
  }
}

// ---- base64 uploads (gRPC) ------------------------------------------------
// The gRPC transport ships each tensor as base64(pickle(tensor))
// (federatedscope/core/message.py:8-9,110-124) and the server decodes it on
// the host (core/auxiliaries/utils.py:95-105, param2tensor).  Here the host
// reads only the pickle framing (core/compression/b64wire.py) and sends the
// base64 text of the storage bytes; this kernel decodes it straight into
// the client's fp32 row.
//
// `src` of a FSAGG_WIRE_B64_F32 segment is a byte offset in the DECODED
// image of `text`: decoded byte d is one of the three bytes of the 4-char
// group at text + 4*(d/3).  Each thread emits 3 fp32 (12 decoded bytes, at
// most 5 groups); the byte phase src % 3 is uniform per segment, so the
// byte shuffle is a compile-time pattern (three instantiations).
constexpr int kB64Elems = 3;

__device__ __forceinline__ uint32_t b64_sextet(uint32_t c, uint32_t &bad) {
  const uint32_t up = c - 'A', lo = c - 'a', dg = c - '0';
  const uint32_t v = up < 26u   ? up
                     : lo < 26u ? lo + 26u
                     : dg < 10u ? dg + 52u
                     : c == '+' ? 62u
                     : c == '/' ? 63u
                                : 64u;
  bad |= v >> 6;
  return v & 63u;
}

// 4 chars (little-endian in x) -> 24 bits, first decoded byte in 23..16
__device__ __forceinline__ uint32_t b64_group(uint32_t x, uint32_t &bad) {
  return (b64_sextet(x & 255u, bad) << 18) |
         (b64_sextet((x >> 8) & 255u, bad) << 12) |
         (b64_sextet((x >> 16) & 255u, bad) << 6) |
         b64_sextet(x >> 24, bad);
}

template <int K>
__device__ __forceinline__ uint32_t b64_byte(const uint32_t (&g)[5]) {
  return (g[K / 3] >> (16 - 8 * (K % 3))) & 255u;
}

template <int K>
__device__ __forceinline__ float b64_word(const uint32_t (&g)[5]) {
  return __uint_as_float(b64_byte<K>(g) | (b64_byte<K + 1>(g) << 8) |
                         (b64_byte<K + 2>(g) << 16) |
                         (b64_byte<K + 3>(g) << 24));
}

template <int S>
__device__ __forceinline__ void b64_emit(const uint32_t (&g)[5], float *o,
                                         int ne) {
  static_assert(kB64Elems == 3, "b64_emit writes three words");
  o[0] = b64_word<S>(g);
  if (ne > 1) o[1] = b64_word<S + 4>(g);
  if (ne > 2) o[2] = b64_word<S + 8>(g);
}

// grid = (ceil(max_len / (kBlock * 3)), nseg).  Segments live on the
// device, so each block checks its own against the decoded extent of
// `text` and the row; a bad segment or a non-alphabet character in a group
// it decodes sets *status (2 / 1) instead of faulting or being silently
// wrong — the host raises on it.
__global__ __launch_bounds__(kBlock) void b64_unpack_kernel(
    const uint32_t *__restrict__ text, int64_t text_groups,
    const WireSeg *__restrict__ segs, int64_t out_len,
    float *__restrict__ out, uint32_t *__restrict__ status) {
  const WireSeg sg = segs[blockIdx.y];
  const int64_t e0 =
      (int64_t(blockIdx.x) * kBlock + threadIdx.x) * kB64Elems;
  if (e0 >= sg.len) return;
  const int64_t cap = 3 * text_groups;  // decoded bytes
  const bool zero = sg.kind == FSAGG_WIRE_ZERO;
  if (sg.len < 0 || sg.dst < 0 || sg.dst > out_len ||
      sg.len > out_len - sg.dst ||
      (!zero && (sg.kind != FSAGG_WIRE_B64_F32 || sg.src < 0 ||
                 sg.src > cap || sg.len > (cap - sg.src) / 4))) {
    status[0] = 2u;
    return;
  }
  float *o = out + sg.dst + e0;
  const int ne = int(min(int64_t(kB64Elems), sg.len - e0));
  if (zero) {
#pragma unroll
    for (int e = 0; e < kB64Elems; ++e)
      if (e < ne) o[e] = 0.0f;
    return;
  }
  const int64_t d = sg.src + 4 * e0;
  const int s = int(sg.src % 3);
  const int64_t g0 = d / 3;
  const int ng = (s + 4 * ne + 2) / 3;
  uint32_t g[5], bad = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j)
    g[j] = j < ng ? b64_group(gld(text + g0 + j), bad) : 0u;
  if (bad) status[0] = 1u;
  if (s == 0)
    b64_emit<0>(g, o, ne);
  else if (s == 1)
    b64_emit<1>(g, o, ne);
  else
    b64_emit<2>(g, o, ne);
}

// numpy's float64 remainder (npy_divmod): the result takes the divisor's
// sign; an exact zero becomes +0.0 for a positive divisor.
__device__ __forceinline__ double py_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0.0) != (m < 0.0)) m = __dadd_rn(m, b);
  } else {
    m = copysign(0.0, b);
  }
  return m;
}

typedef long long ll2v __attribute__((ext_vector_type(2)));
typedef double d2v __attribute__((ext_vector_type(2)));

// Two consecutive elements per lane (16-B non-temporal loads of every share
// row), rows taken eight at a time so their loads are in flight together;
// the adds stay in list order.  100 × 6M int64 shares: 0.786 ms against
// 0.833–0.844 for four rows and plain loads (profiles/r06/ss_rows8_nt.jsonl;
// sixteen rows 0.878, rejected/ss_rows16_nt.jsonl).
__device__ __forceinline__ void ss_load2(const void *row, bool is_int,
                                         int64_t p, bool two, double &x0,
                                         double &x1) {
  if (is_int) {
    const int64_t *r = static_cast<const int64_t *>(row) + p;
    if (two) {
      const ll2v v = gld_nt(reinterpret_cast<const ll2v *>(r));
      x0 = __ll2double_rn(v.x);
      x1 = __ll2double_rn(v.y);
    } else {
      x0 = __ll2double_rn(gld(r));
      x1 = 0.0;
    }
  } else {
    const double *r = static_cast<const double *>(row) + p;
    if (two) {
      const d2v v = gld_nt(reinterpret_cast<const d2v *>(r));
      x0 = v.x;
      x1 = v.y;
    } else {
      x0 = gld(r);
      x1 = 0.0;
    }
  }
}

__device__ __forceinline__ float ss_recover_one(double acc, double mod,
                                                double maximum, double epsilon,
                                                double total) {
  // _fixedpoint2float: x %= mod; x > maximum ? -(mod - x)/eps : x/eps
  const double x = py_mod(acc, mod);
  const double r = x > maximum ? -__ddiv_rn(__dsub_rn(mod, x), epsilon)
                               : __ddiv_rn(x, epsilon);
  // avg /= training_set_size; torch.FloatTensor(avg)
  return __double2float_rn(__ddiv_rn(r, total));
}

__global__ __launch_bounds__(kBlock) void ss_recover_kernel(
    const void *const *__restrict__ rows, const uint8_t *__restrict__ is_int,
    int n, int64_t numel, double weight, double mod, double maximum,
    double epsilon, double total, int recover, float *__restrict__ out,
    double *__restrict__ out_sum) {
  const int64_t p = 2 * (int64_t(blockIdx.x) * kBlock + threadIdx.x);
  if (p >= numel) return;
  const bool two = p + 1 < numel;
  // avg = x_0 * w, then avg += x_i * w in list order (float64; w = 1.0, or
  // 1/n with ignore_weight — x * 1.0 is exact)
  double a0 = 0.0, a1 = 0.0;
  int i = 0;
  for (; i + kSsRows <= n; i += kSsRows) {
    double x[kSsRows][2];
#pragma unroll
    for (int u = 0; u < kSsRows; ++u)
      ss_load2(rows[i + u], is_int[i + u], p, two, x[u][0], x[u][1]);
#pragma unroll
    for (int u = 0; u < kSsRows; ++u) {
      const double y0 = __dmul_rn(x[u][0], weight);
      const double y1 = __dmul_rn(x[u][1], weight);
      a0 = (i + u == 0) ? y0 : __dadd_rn(a0, y0);
      a1 = (i + u == 0) ? y1 : __dadd_rn(a1, y1);
    }
  }
  for (; i < n; ++i) {
    double x0, x1;
    ss_load2(rows[i], is_int[i], p, two, x0, x1);
    x0 = __dmul_rn(x0, weight);
    x1 = __dmul_rn(x1, weight);
    a0 = i == 0 ? x0 : __dadd_rn(a0, x0);
    a1 = i == 0 ? x1 : __dadd_rn(a1, x1);
  }
  if (!recover) {
    out_sum[p] = a0;
    if (two) out_sum[p + 1] = a1;
    return;
  }
  out[p] = ss_recover_one(a0, mod, maximum, epsilon, total);
  if (two) out[p + 1] = ss_recover_one(a1, mod, maximum, epsilon, total);
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_wire_unpack_f32(const void *src, int64_t src_bytes,
                                     const void *segs, const float *scales,
                                     int nscale, int nseg, int64_t max_len,
                                     float *out, int64_t out_len,
                                     fsagg_stream_t stream) {
  if (!src || !segs || !out || nseg < 0 || max_len < 0 || src_bytes < 0 ||
      out_len < 0 || nscale < 0 || (nscale > 0 && !scales)) {
    set_error("fsagg_wire_unpack_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (nseg == 0 || max_len == 0) return FSAGG_OK;
  if (nseg > 65535) {
    set_error("fsagg_wire_unpack_f32: %d segments > 65535", nseg);
    return FSAGG_EINVAL;
  }
  const int64_t per = int64_t(kBlock) * kPerThread;
  hipLaunchKernelGGL(wire_unpack_kernel,
                     dim3(unsigned((max_len + per - 1) / per), unsigned(nseg)),
                     dim3(kBlock), 0, as_stream(stream),
                     static_cast<const unsigned char *>(src),
                     static_cast<const WireSeg *>(segs), scales, nscale,
                     src_bytes, out_len, out);
  return check_launch("fsagg_wire_unpack_f32");
}

extern "C" int fsagg_b64_unpack_f32(const void *text, int64_t text_bytes,
                                    const void *segs, int nseg,
                                    int64_t max_len, float *out,
                                    int64_t out_len, uint32_t *status,
                                    fsagg_stream_t stream) {
  if (!text || !segs || !out || !status || nseg < 0 || max_len < 0 ||
      text_bytes < 0 || out_len < 0 || text_bytes % 4 ||
      reinterpret_cast<uintptr_t>(text) % 4) {
    set_error("fsagg_b64_unpack_f32: invalid argument (text must be "
              "4-byte aligned whole 4-char groups)");
    return FSAGG_EINVAL;
  }
  if (nseg == 0 || max_len == 0) return FSAGG_OK;
  if (nseg > 65535) {
    set_error("fsagg_b64_unpack_f32: %d segments > 65535", nseg);
    return FSAGG_EINVAL;
  }
  const int64_t per = int64_t(kBlock) * kB64Elems;
  hipLaunchKernelGGL(b64_unpack_kernel,
                     dim3(unsigned((max_len + per - 1) / per), unsigned(nseg)),
                     dim3(kBlock), 0, as_stream(stream),
                     static_cast<const uint32_t *>(text), text_bytes / 4,
                     static_cast<const WireSeg *>(segs), out_len, out,
                     status);
  return check_launch("fsagg_b64_unpack_f32");
}

extern "C" int fsagg_ss_recover_f32(const void *const *rows,
                                    const uint8_t *row_is_int, int n,
                                    int64_t numel, double weight, double mod,
                                    double maximum, double epsilon,
                                    double total, int recover, float *out,
                                    double *out_sum, fsagg_stream_t stream) {
  if (!rows || !row_is_int || n < 1 || numel < 0 ||
      (recover && !out) || (!recover && !out_sum)) {
    set_error("fsagg_ss_recover_f32: invalid argument (n=%d)", n);
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  const int64_t pairs = (numel + 1) / 2;
  hipLaunchKernelGGL(ss_recover_kernel,
                     dim3(unsigned((pairs + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, as_stream(stream), rows, row_is_int, n,
                     numel, weight, mod, maximum, epsilon, total, recover,
                     out, out_sum);
  return check_launch("fsagg_ss_recover_f32");
}
