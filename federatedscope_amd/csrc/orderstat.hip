// Coordinate-wise order statistics over client buckets (gfx950):
// median (median_aggregator.py:43-52) and trimmed mean
// (trimmedmean_aggregator.py:44-57, Bulyan's stage 2 bulyan_aggregator.py:92-105).
//
// One lane owns one coordinate (column of the n×P client stack).  The lane
// loads its n values with coalesced 4-B loads (64 consecutive coordinates per
// wave-instruction, one row at a time), maps them to order-preserving uint32
// keys and sorts them in registers with a bitonic network that is generated
// at compile time as straight-line min/max code (NMAX ∈ {4..256}; padding
// keys 0xFFFFFFFF sort last) for n <= 64.  For 64 < n <= 256 the keys stay
// in registers and the two needed ranks are found together by a 32-step
// radix (bit-by-bit) select — branch-free counting over the register file;
// the straight-line bitonic network beyond 64 keys is too large for the
// compiler.  n > 256 uses the same radix select re-reading the column from
// L2.
//
// Algorithmic bytes per coordinate: 4·n read + 4 (base) read + 4 written.
#include <utility>

#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;
constexpr uint32_t kPad = 0xFFFFFFFFu;

// ---- compile-time bitonic network --------------------------------------
template <int N, int SIZE, int STRIDE, int I>
__device__ __forceinline__ void cmpx(uint32_t (&k)[N]) {
  constexpr int J = I ^ STRIDE;
  if constexpr (J > I) {
    constexpr bool up = (I & SIZE) == 0;
    const uint32_t a = k[I], b = k[J];
    const uint32_t lo = a < b ? a : b;
    const uint32_t hi = a < b ? b : a;
    k[I] = up ? lo : hi;
    k[J] = up ? hi : lo;
  }
}

template <int N, int SIZE, int STRIDE, int... I>
__device__ __forceinline__ void stage(uint32_t (&k)[N],
                                      std::integer_sequence<int, I...>) {
  (cmpx<N, SIZE, STRIDE, I>(k), ...);
}

template <int N, int SIZE, int STRIDE>
__device__ __forceinline__ void merge_level(uint32_t (&k)[N]) {
  stage<N, SIZE, STRIDE>(k, std::make_integer_sequence<int, N>{});
  if constexpr (STRIDE > 1) merge_level<N, SIZE, STRIDE / 2>(k);
}

template <int N, int SIZE>
__device__ __forceinline__ void sort_from(uint32_t (&k)[N]) {
  merge_level<N, SIZE, SIZE / 2>(k);
  if constexpr (SIZE < N) sort_from<N, SIZE * 2>(k);
}

template <int N>
__device__ __forceinline__ void bitonic_sort(uint32_t (&k)[N]) {
  sort_from<N, 2>(k);
}

// read k[idx] for a runtime idx without dynamic register indexing
template <int N, int... I>
__device__ __forceinline__ uint32_t pick(const uint32_t (&k)[N], int idx,
                                         std::integer_sequence<int, I...>) {
  uint32_t r = 0;
  ((r = (I == idx) ? k[I] : r), ...);
  return r;
}

// Σ key2f(k[j]) for lo <= j < hi, in float64, ascending order
template <int N, int... I>
__device__ __forceinline__ double mid_sum(const uint32_t (&k)[N], int lo,
                                          int hi,
                                          std::integer_sequence<int, I...>) {
  double s = 0.0;
  ((s += (I >= lo && I < hi) ? double(key2f(k[I])) : 0.0), ...);
  return s;
}

// The reference computes cat([T, -top_k, -bottom_k]).sum(): for a column that
// holds ±inf/NaN with k >= 1 an infinity is always among the excluded values,
// so the fp32 sum is inf - inf = NaN; with k == 0 it is Σall (inf or NaN).
template <int N, int... I>
__device__ __forceinline__ float nonfinite_sum(const uint32_t (&k)[N], int n,
                                               int kk, bool nan,
                                               std::integer_sequence<int, I...>) {
  if (kk > 0 || nan) return __builtin_nanf("");
  float s = 0.0f;
  ((s = (I < n) ? add_rn(s, key2f(k[I])) : s), ...);
  return s;
}

enum Mode { kMedian = 0, kTrimmed = 1 };

// Load a lane's column of n values into N key registers (pads = kPad).
// Branch-free on purpose: rows past n re-read row n-1 (an L1/L2 hit) and are
// masked to kPad, so all N loads issue back to back and the wave waits once
// — a per-row `if (j < n)` splits the loop into N basic blocks and every
// load then waits out its own HBM round trip.
template <int N>
__device__ __forceinline__ void load_column(const float *const *rows, int n,
                                            int64_t p, uint32_t (&k)[N],
                                            bool &nan, bool &nonfinite) {
  float x[N];
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = rows[j < n ? j : n - 1][p];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const bool real = j < n;
    nan |= real && __builtin_isnan(x[j]);
    nonfinite |= real && !__builtin_isfinite(x[j]);
    k[j] = real ? f2key(x[j]) : kPad;
  }
}

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_reg_kernel(
    const float *const *__restrict__ rows, int n, int64_t numel, int kk,
    float divisor, const float *__restrict__ base, float *__restrict__ out) {
  const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= numel) return;
  uint32_t k[N];
  bool nan = false, nonfinite = false;
  load_column<N>(rows, n, p, k, nan, nonfinite);
  bitonic_sort<N>(k);
  using Seq = std::make_integer_sequence<int, N>;
  float r;
  if constexpr (MODE == kMedian) {
    const float lo = key2f(pick<N>(k, (n - 1) / 2, Seq{}));
    const float hi = key2f(pick<N>(k, n / 2, Seq{}));
    // (median(T) - median(-T)) / 2, literally
    r = __fdiv_rn(lo - (-hi), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    float s;
    if (!nonfinite) {
      s = float(mid_sum<N>(k, kk, n - kk, Seq{}));
    } else {
      s = nonfinite_sum<N>(k, n, kk, nan, Seq{});
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(base[p], r);
  out[p] = r;
}

// ---- 64 < n <= 256: register-resident radix select ----------------------
template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_radix_kernel(
    const float *const *__restrict__ rows, int n, int64_t numel, int kk,
    float divisor, const float *__restrict__ base, float *__restrict__ out) {
  const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= numel) return;
  uint32_t k[N];
  bool nan = false, nonfinite = false;
  load_column<N>(rows, n, p, k, nan, nonfinite);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;
  // p = the key of rank r: the largest prefix with #(key <= prefix|lowbits) <= r
  uint32_t p1 = 0, p2 = 0;
#pragma unroll 1
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t m = (1u << bit) - 1u;
    const uint32_t c1 = p1 | m, c2 = p2 | m;
    int n1 = 0, n2 = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      n1 += k[j] <= c1;
      n2 += k[j] <= c2;
    }
    if (n1 <= r1) p1 |= 1u << bit;
    if (n2 <= r2) p2 |= 1u << bit;
  }
  float r;
  if constexpr (MODE == kMedian) {
    r = __fdiv_rn(key2f(p1) - (-key2f(p2)), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    float s;
    if (!nonfinite) {
      const uint32_t klo = p1, khi = p2;
      int below = 0, eq_lo = 0, inside = 0;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        below += k[j] < klo;
        eq_lo += k[j] == klo;
        const bool in = k[j] > klo && k[j] < khi;
        inside += in;
        acc += in ? double(key2f(k[j])) : 0.0;
      }
      const int keep = n - 2 * kk;
      if (klo == khi) {
        acc = double(key2f(klo)) * keep;
      } else {
        const int lo_kept = min(below + eq_lo, n - kk) - kk;
        const int hi_kept = keep - lo_kept - inside;
        acc += double(key2f(klo)) * lo_kept + double(key2f(khi)) * hi_kept;
      }
      s = float(acc);
    } else if (kk > 0 || nan) {
      s = __builtin_nanf("");
    } else {
      s = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) s = j < n ? add_rn(s, key2f(k[j])) : s;
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(base[p], r);
  out[p] = r;
}

// ---- 64 < n <= 255: LDS byte-histogram radix select ----------------------
// Keys stay in registers (one lane = one coordinate).  A rank is found in 4
// passes of 8 bits: each pass adds the lane's matching keys into a private
// 256-bin histogram of byte counters in LDS (ds_add_u32 of 1 << 8·(d & 3)
// into word d / 4; n <= 255 keeps every byte from overflowing), then the lane
// scans its 64 words (v_sad_u8 sums four bins per word) for the bin that
// holds the rank.  ≈ 4·(3n + 400) VALU per rank instead of the 2·32·n of the
// bit-by-bit select.  Histogram words are laid out [word][lane], so the 64
// lanes of a wave always hit 64 distinct banks.
constexpr int kHistWords = 64;                   // 256 byte bins per lane
constexpr int kHistLds = 4 * kHistWords * kWave; // 4 waves: 64 KiB

__device__ __forceinline__ void hist_clear(uint32_t *H) {
#pragma unroll
  for (int w = 0; w < kHistWords; ++w) H[w * kWave] = 0u;
}

template <int N>
__device__ __forceinline__ void hist_add(uint32_t *H, const uint32_t (&k)[N],
                                         int n, uint32_t mask, uint32_t prefix,
                                         int shift) {
  // Pads (kPad, the largest key) may be counted: they sort after every
  // real key and ranks are < n.  Only N = 256 must skip them — a bin could
  // then reach 256 and overflow its byte.
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (N == 256 && j >= n) continue;
    const uint32_t key = k[j];
    if ((key & mask) == prefix) {
      const uint32_t d = (key >> shift) & 255u;
      atomicAdd(&H[(d >> 2) * kWave], 1u << ((d & 3u) * 8u));
    }
  }
}

// Bin (0..255) holding rank r of the histogram, and the count below it.
__device__ __forceinline__ uint32_t hist_scan(const uint32_t *H, int r,
                                             int &below) {
  int cum = 0, fcum = 0;
  uint32_t fw = 0, fx = 0;
  bool found = false;
#pragma unroll 8
  for (int w = 0; w < kHistWords; ++w) {
    const uint32_t x = H[w * kWave];
    const int s = int(__builtin_amdgcn_sad_u8(x, 0u, 0u));
    const bool here = !found && cum + s > r;
    fw = here ? uint32_t(w) : fw;
    fx = here ? x : fx;
    fcum = here ? cum : fcum;
    found |= here;
    cum += s;
  }
  uint32_t byte = 3;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int c = int((fx >> (8 * b)) & 255u);
    const bool stop = byte == 3 && fcum + c > r;
    byte = stop ? uint32_t(b) : byte;
    fcum += (byte == 3) ? c : 0;
  }
  below = fcum;
  return fw * 4 + byte;
}

// Refine rank r below a first-pass bin d0 (passes 2..4).
template <int N>
__device__ __forceinline__ uint32_t hist_refine(uint32_t *H,
                                               const uint32_t (&k)[N], int n,
                                               uint32_t d0, int r) {
  uint32_t prefix = d0 << 24;
#pragma unroll 1
  for (int pass = 1; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t mask = 0xFFFFFFFFu << (shift + 8);
    hist_clear(H);
    hist_add<N>(H, k, n, mask, prefix, shift);
    int below;
    const uint32_t d = hist_scan(H, r, below);
    r -= below;
    prefix |= d << shift;
  }
  return prefix;
}

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_hist_kernel(
    const float *const *__restrict__ rows, int n, int64_t numel, int kk,
    float divisor, const float *__restrict__ base, float *__restrict__ out) {
  __shared__ uint32_t hist[kHistLds];
  uint32_t *H = hist + (threadIdx.x / kWave) * kHistWords * kWave +
                (threadIdx.x & (kWave - 1));
  const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  const bool live = p < numel;
  uint32_t k[N];
  bool nan = false, nonfinite = false;
  load_column<N>(rows, n, live ? p : 0, k, nan, nonfinite);
  // pass 1 is shared by both ranks
  hist_clear(H);
  hist_add<N>(H, k, n, 0u, 0u, 24);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;
  int b1, b2;
  const uint32_t d1 = hist_scan(H, r1, b1);
  const uint32_t d2 = hist_scan(H, r2, b2);
  const uint32_t k1 = hist_refine<N>(H, k, n, d1, r1 - b1);
  uint32_t k2;
  if (MODE == kMedian) {
    // the upper middle is k1 itself or the smallest key above it
    int le = 0;
    uint32_t above = kPad;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j < n) {
        le += k[j] <= k1;
        above = k[j] > k1 && k[j] < above ? k[j] : above;
      }
    }
    k2 = le > r2 ? k1 : above;
  } else {
    k2 = hist_refine<N>(H, k, n, d2, r2 - b2);
  }
  if (!live) return;
  float r;
  if constexpr (MODE == kMedian) {
    r = __fdiv_rn(key2f(k1) - (-key2f(k2)), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    float s;
    if (!nonfinite) {
      int below = 0, eq_lo = 0, inside = 0;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j < n) {
          below += k[j] < k1;
          eq_lo += k[j] == k1;
          const bool in = k[j] > k1 && k[j] < k2;
          inside += in;
          acc += in ? double(key2f(k[j])) : 0.0;
        }
      }
      const int keep = n - 2 * kk;
      if (k1 == k2) {
        acc = double(key2f(k1)) * keep;
      } else {
        const int lo_kept = min(below + eq_lo, n - kk) - kk;
        const int hi_kept = keep - lo_kept - inside;
        acc += double(key2f(k1)) * lo_kept + double(key2f(k2)) * hi_kept;
      }
      s = float(acc);
    } else if (kk > 0 || nan) {
      s = __builtin_nanf("");
    } else {
      s = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) s = j < n ? add_rn(s, key2f(k[j])) : s;
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(base[p], r);
  out[p] = r;
}

// ---- generic n: radix select (binary search on the key bits) -----------
__device__ __forceinline__ uint32_t select_rank(const float *const *rows,
                                                int n, int64_t p, int rank) {
  // smallest key v such that #(key <= v) > rank
  uint32_t prefix = 0;
  for (int bit = 31; bit >= 0; --bit) {
    const uint32_t cand = prefix | ((1u << bit) - 1u);  // all lower bits set
    int cnt = 0;
    for (int j = 0; j < n; ++j) cnt += f2key(rows[j][p]) <= cand;
    if (cnt <= rank) prefix |= 1u << bit;
  }
  return prefix;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_generic_kernel(
    const float *const *__restrict__ rows, int n, int64_t numel, int kk,
    float divisor, const float *__restrict__ base, float *__restrict__ out) {
  const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= numel) return;
  bool nan = false, nonfinite = false;
  for (int j = 0; j < n; ++j) {
    const float x = rows[j][p];
    nan |= __builtin_isnan(x);
    nonfinite |= !__builtin_isfinite(x);
  }
  float r;
  if constexpr (MODE == kMedian) {
    const float lo = key2f(select_rank(rows, n, p, (n - 1) / 2));
    const float hi = key2f(select_rank(rows, n, p, n / 2));
    r = __fdiv_rn(lo - (-hi), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    const uint32_t klo = select_rank(rows, n, p, kk);
    const uint32_t khi = select_rank(rows, n, p, n - kk - 1);
    float s;
    if (!nonfinite) {
      // kept ranks [kk, n-kk): strictly inside (klo, khi) plus tie copies
      double acc = 0.0;
      int below = 0, eq_lo = 0, inside = 0;
      for (int j = 0; j < n; ++j) {
        const float x = rows[j][p];
        const uint32_t key = f2key(x);
        below += key < klo;
        eq_lo += key == klo;
        const bool in = key > klo && key < khi;
        inside += in;
        if (in) acc += double(x);
      }
      const int keep = n - 2 * kk;
      if (klo == khi) {
        acc = double(key2f(klo)) * keep;
      } else {
        const int lo_kept = min(below + eq_lo, n - kk) - kk;
        const int hi_kept = keep - lo_kept - inside;
        acc += double(key2f(klo)) * lo_kept + double(key2f(khi)) * hi_kept;
      }
      s = float(acc);
    } else {
      // Σall − Σtop − Σbottom in fp32: with k >= 1 an infinity is always
      // among the excluded values, so inf - inf (or a NaN) gives NaN;
      // with k == 0 the result is Σall itself.
      float all = 0.0f;
      for (int j = 0; j < n; ++j) all = add_rn(all, rows[j][p]);
      s = (kk == 0 && !nan) ? all : __builtin_nanf("");
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(base[p], r);
  out[p] = r;
}

template <int MODE>
int launch(const float *const *rows, int n, int64_t numel, int kk,
           float divisor, const float *base, float *out, hipStream_t s) {
  const unsigned grid = unsigned((numel + kBlock - 1) / kBlock);
#define FSAGG_OS(NN)                                                        \
  hipLaunchKernelGGL((orderstat_reg_kernel<NN, MODE>), dim3(grid),         \
                     dim3(kBlock), 0, s, rows, n, numel, kk, divisor, base, \
                     out)
  if (n <= 4) FSAGG_OS(4);
  else if (n <= 8) FSAGG_OS(8);
  else if (n <= 16) FSAGG_OS(16);
  else if (n <= 32) FSAGG_OS(32);
  else if (n <= 64) FSAGG_OS(64);
#define FSAGG_RX(NN)                                                        \
  hipLaunchKernelGGL((orderstat_hist_kernel<NN, MODE>), dim3(grid),        \
                     dim3(kBlock), 0, s, rows, n, numel, kk, divisor, base, \
                     out)
  else if (n <= 96) FSAGG_RX(96);
  else if (n <= 128) FSAGG_RX(128);
  else if (n <= 160) FSAGG_RX(160);
  else if (n <= 192) FSAGG_RX(192);
  else if (n <= 224) FSAGG_RX(224);
  else if (n <= 255) FSAGG_RX(256);
  else
    hipLaunchKernelGGL((orderstat_generic_kernel<MODE>), dim3(grid),
                       dim3(kBlock), 0, s, rows, n, numel, kk, divisor, base,
                       out);
#undef FSAGG_OS
#undef FSAGG_RX
  return check_launch(MODE == kMedian ? "fsagg_coord_median_f32"
                                      : "fsagg_trimmed_mean_f32");
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_coord_median_f32(const float *const *rows, int n,
                                      int64_t numel, const float *base,
                                      float *out, fsagg_stream_t stream) {
  if (!rows || !out || n < 1 || numel < 0) {
    set_error("fsagg_coord_median_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  return launch<kMedian>(rows, n, numel, 0, 2.0f, base, out,
                         as_stream(stream));
}

extern "C" int fsagg_trimmed_mean_f32(const float *const *rows, int n,
                                      int64_t numel, int k, float divisor,
                                      const float *base, float *out,
                                      fsagg_stream_t stream) {
  if (!rows || !out || n < 1 || numel < 0 || k < 0 || 2 * k >= n) {
    set_error("fsagg_trimmed_mean_f32: invalid argument (n=%d k=%d)", n, k);
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  return launch<kTrimmed>(rows, n, numel, k, divisor, base, out,
                          as_stream(stream));
}
