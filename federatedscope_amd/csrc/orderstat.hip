// Coordinate-wise order statistics over client buckets (gfx950):
// median (median_aggregator.py:43-52) and trimmed mean
// (trimmedmean_aggregator.py:44-57, Bulyan's stage 2 bulyan_aggregator.py:92-105).
//
// One lane owns one coordinate (column of the n×P client stack).  The lane
// loads its n values with coalesced 4-B loads (64 consecutive coordinates per
// wave-instruction, one row at a time) and maps them to order-preserving
// uint32 keys.
//  - n <= 32 and 56 < n <= 64: the keys are sorted in registers by a sorting
//    network generated at compile time as straight-line min/max code
//    (padding keys 0xFFFFFFFF sort last).
//  - 32 < n <= 56 and 64 < n <= 255: range-adaptive radix select + LDS
//    compaction (orderstat_select.hip, one translation unit per
//    register-array size).
//  - 255 < n <= 65535: the same select streaming the column from memory in
//    each pass (orderstat_stream.hip).
//  - more than 65535 clients or 2^30 columns: bit-by-bit radix select that
//    re-reads the column 64 times.
//
// Algorithmic bytes per coordinate: 4·n read + 4 (base) read + 4 written.
#include <atomic>

#include "orderstat.h"

namespace fsagg {
namespace os {
namespace {

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
  for (int j = 0; j < N; ++j) x[j] = gld_nt(rows[j < n ? j : n - 1] + p);
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
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  const BlockRows br = block_rows(rs, blockIdx.x);
  if (int(threadIdx.x) >= br.len) return;
  const int64_t p = br.lo + threadIdx.x;
  const float *__restrict__ base = br.base;
  uint32_t k[N];
  bool nan = false, nonfinite = false;
  // the init coordinate with the column, not after the sort (its latency
  // would be exposed at the end of every wave)
  const float bval = base ? gld_nt(base + p) : 0.0f;
  load_column<N>(br.rows, n, p, k, nan, nonfinite);
  if constexpr (MODE == kMedian) {
    // the two middle positions of every n this size serves: n <= 4 at
    // N = 4, N/2 < n <= N otherwise, and 32 < n <= 64 at N = 64 (launch)
    constexpr int lo = N <= 4 ? 0 : (N == 64 ? 16 : N / 4);
    select_network<N, lo, N / 2>(k);
  } else {
    sort_network<N>(k);
  }
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
  if (base) r = add_rn(bval, r);
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
    for (int j = 0; j < n; ++j) cnt += f2key(gld(rows[j] + p)) <= cand;
    if (cnt <= rank) prefix |= 1u << bit;
  }
  return prefix;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_generic_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  const BlockRows br = block_rows(rs, blockIdx.x);
  if (int(threadIdx.x) >= br.len) return;
  const int64_t p = br.lo + threadIdx.x;
  const float *const *__restrict__ rows = br.rows;
  const float *__restrict__ base = br.base;
  bool nan = false, nonfinite = false;
  for (int j = 0; j < n; ++j) {
    const float x = gld(rows[j] + p);
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
        const float x = gld(rows[j] + p);
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
      for (int j = 0; j < n; ++j) all = add_rn(all, gld(rows[j] + p));
      s = (kk == 0 && !nan) ? all : __builtin_nanf("");
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(gld(base + p), r);
  out[p] = r;
}

// Clients from which 64 < n <= 255 takes the two-wave kernel;
// fsagg_orderstat_set_pair_min() moves it for A/B measurements.
std::atomic<int> g_pair_min{kPairMinDefault};
// The client range [lo, hi] of 255 < n that takes the K-wave kernel
// (orderstat_group.h), per mode (median, trimmed mean), from interleaved
// A/B against the two-pass streaming kernel at 5.3 GB
// (profiles/r05/orderstat_group_ab.jsonl): the median gains from n = 384
// (n = 500: 1.21 against 1.50 ms) and loses at n = 300 (1.56 / 1.47); the
// trimmed mean's serial list tail in wave 0 keeps it behind (n = 500:
// 1.94 / 1.88), so it streams.  fsagg_orderstat_set_group_max() opens the
// whole range to both modes for tests and A/B.
constexpr int kGroupDefault[2][2] = {{384, 512}, {513, 512}};
std::atomic<int> g_group[2][2] = {{{kGroupDefault[0][0]},
                                   {kGroupDefault[0][1]}},
                                  {{kGroupDefault[1][0]},
                                   {kGroupDefault[1][1]}}};

template <int MODE>
int launch(const RowSrc &rs, int nchunk, int n, int kk, float divisor,
           float *out, hipStream_t s) {
  const unsigned grid = rows_grid(rs, nchunk);
#define FSAGG_OS(NN)                                                        \
  hipLaunchKernelGGL((orderstat_reg_kernel<NN, MODE>), dim3(grid),         \
                     dim3(kBlock), 0, s, rs, n, kk, divisor, out)
  if (n <= 4) FSAGG_OS(4);
  else if (n <= 8) FSAGG_OS(8);
  else if (n <= 16) FSAGG_OS(16);
  else if (n <= 32) FSAGG_OS(32);
  // 33..56: the select kernel (n = 50: median −6 %, trimmed −11 % against
  // the 64-key sort); 57..64 the sort (n = 64: equal or 4 % faster)
  else if (n <= 64 && (n > 56 || rs.numel > (int64_t(1) << 30)))
    FSAGG_OS(64);
#define FSAGG_SEL(NN)                                                       \
  if (pair)                                                                \
    launch_pair<NN / 2, MODE>(rs, pgrid, n, kk, divisor, out, s);          \
  else                                                                     \
    launch_select<NN, MODE>(rs, grid, n, kk, divisor, out, s)
  else if (n <= 255 && rs.numel <= (int64_t(1) << 30) &&
           n >= g_group[MODE == kMedian ? 0 : 1][0].load() &&
           n <= g_group[MODE == kMedian ? 0 : 1][1].load() &&
           launch_group<MODE>(rs, rs.chunks ? unsigned(nchunk) * 4u
                                            : unsigned((rs.numel + kWave - 1) /
                                                       kWave),
                              n, kk, divisor, out, s)) {
    // the K-wave kernel, where a tuning hook opened it below 256 clients
  } else if (n <= 255 && rs.numel <= (int64_t(1) << 30)) {
    // the two-wave form from g_pair_min clients up (orderstat_pair.h)
    const bool pair = n >= g_pair_min.load(std::memory_order_relaxed);
    const unsigned pgrid = rs.chunks ? unsigned(nchunk) * 4u
                                     : unsigned((rs.numel + kWave - 1) / kWave);
    switch ((n + kSelStep - 1) / kSelStep * kSelStep) {
    case 40: FSAGG_SEL(40); break;
    case 48: FSAGG_SEL(48); break;
    case 56: FSAGG_SEL(56); break;
    case 72: FSAGG_SEL(72); break;
    case 80: FSAGG_SEL(80); break;
    case 88: FSAGG_SEL(88); break;
    case 96: FSAGG_SEL(96); break;
    case 104: FSAGG_SEL(104); break;
    case 112: FSAGG_SEL(112); break;
    case 120: FSAGG_SEL(120); break;
    case 128: FSAGG_SEL(128); break;
    case 136: FSAGG_SEL(136); break;
    case 144: FSAGG_SEL(144); break;
    case 152: FSAGG_SEL(152); break;
    case 160: FSAGG_SEL(160); break;
    case 168: FSAGG_SEL(168); break;
    case 176: FSAGG_SEL(176); break;
    case 184: FSAGG_SEL(184); break;
    case 192: FSAGG_SEL(192); break;
    case 200: FSAGG_SEL(200); break;
    case 208: FSAGG_SEL(208); break;
    case 216: FSAGG_SEL(216); break;
    case 224: FSAGG_SEL(224); break;
    case 232: FSAGG_SEL(232); break;
    case 240: FSAGG_SEL(240); break;
    case 248: FSAGG_SEL(248); break;
    case 256: FSAGG_SEL(256); break;
    }
  } else if (n <= 65535 && rs.numel <= (int64_t(1) << 30)) {
    // one HBM pass with the column split over a workgroup's waves, up to
    // n = 512 (g_group_max moves it for A/B); the streaming kernel above
    const unsigned ggrid = rs.chunks ? unsigned(nchunk) * 4u
                                     : unsigned((rs.numel + kWave - 1) / kWave);
    const std::atomic<int> *rg = g_group[MODE == kMedian ? 0 : 1];
    if (n < rg[0].load(std::memory_order_relaxed) ||
        n > rg[1].load(std::memory_order_relaxed) ||
        !launch_group<MODE>(rs, ggrid, n, kk, divisor, out, s))
      launch_stream<MODE>(rs, grid, n, kk, divisor, out, s);
  } else {
    hipLaunchKernelGGL((orderstat_generic_kernel<MODE>), dim3(grid),
                       dim3(kBlock), 0, s, rs, n, kk, divisor, out);
  }
#undef FSAGG_OS
#undef FSAGG_SEL
  return check_launch(MODE == kMedian ? "coordinate median"
                                      : "trimmed mean");
}

RowSrc flat_src(const float *const *rows, int64_t numel, const float *base) {
  return RowSrc{rows, 0, nullptr, numel, base, nullptr, 0};
}

// the row-set entry points' shared argument checks
bool rows_args_ok(const fsagg_rows *rows, const fsagg_chunk *chunks,
                  int nchunk, int64_t numel, int64_t base_ss, float *out,
                  const char *what) {
  if (!rows || !rows->tab || rows->n < 1 || rows->nseg < 1 || !out ||
      nchunk < 0 || (nchunk > 0 && !chunks) || numel < 0 || base_ss < 0) {
    set_error("%s: invalid argument", what);
    return false;
  }
  return true;
}

}  // namespace
}  // namespace os
}  // namespace fsagg

using namespace fsagg;
using namespace fsagg::os;

extern "C" int fsagg_coord_median_f32(const float *const *rows, int n,
                                      int64_t numel, const float *base,
                                      float *out, fsagg_stream_t stream) {
  if (!rows || !out || n < 1 || numel < 0) {
    set_error("fsagg_coord_median_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  return launch<kMedian>(flat_src(rows, numel, base), 0, n, 0, 2.0f, out,
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
  return launch<kTrimmed>(flat_src(rows, numel, base), 0, n, k, divisor, out,
                          as_stream(stream));
}

extern "C" int fsagg_coord_median_rows_f32(const fsagg_rows *rows,
                                           const fsagg_chunk *chunks,
                                           int nchunk, int64_t numel,
                                           const float *const *base,
                                           int64_t base_ss, float *out,
                                           fsagg_stream_t stream) {
  if (!rows_args_ok(rows, chunks, nchunk, numel, base_ss, out,
                    "fsagg_coord_median_rows_f32"))
    return FSAGG_EINVAL;
  if (nchunk == 0) return FSAGG_OK;
  const RowSrc rs{rows->tab, rows->ss, chunks, numel, nullptr, base,
                  base_ss};
  return launch<kMedian>(rs, nchunk, rows->n, 0, 2.0f, out,
                         as_stream(stream));
}

extern "C" int fsagg_trimmed_mean_rows_f32(const fsagg_rows *rows,
                                           const fsagg_chunk *chunks,
                                           int nchunk, int64_t numel, int k,
                                           float divisor,
                                           const float *const *base,
                                           int64_t base_ss, float *out,
                                           fsagg_stream_t stream) {
  if (!rows_args_ok(rows, chunks, nchunk, numel, base_ss, out,
                    "fsagg_trimmed_mean_rows_f32"))
    return FSAGG_EINVAL;
  if (k < 0 || 2 * k >= rows->n) {
    set_error("fsagg_trimmed_mean_rows_f32: invalid k=%d for n=%d", k,
              rows->n);
    return FSAGG_EINVAL;
  }
  if (nchunk == 0) return FSAGG_OK;
  const RowSrc rs{rows->tab, rows->ss, chunks, numel, nullptr, base,
                  base_ss};
  return launch<kTrimmed>(rs, nchunk, rows->n, k, divisor, out,
                          as_stream(stream));
}

extern "C" int fsagg_orderstat_set_pair_min(int n) {
  return g_pair_min.exchange(n < 0 ? kPairMinDefault : n);
}

extern "C" int fsagg_orderstat_set_group_range(int lo, int hi) {
  const int prev = g_group[0][0].load();
  for (int m = 0; m < 2; ++m) {
    g_group[m][0] = lo < 0 ? kGroupDefault[m][0] : lo;
    g_group[m][1] = lo < 0 ? kGroupDefault[m][1] : hi;
  }
  return prev;
}

extern "C" int fsagg_orderstat_set_group_waves(int k) {
  return g_group_waves.exchange(k < 2 || k > 8 ? 8 : k);
}

extern "C" int fsagg_orderstat_set_group_max(int n) {
  const int prev = g_group[0][1].load();
  for (int m = 0; m < 2; ++m) {
    g_group[m][0] = n < 0 ? kGroupDefault[m][0] : 256;
    g_group[m][1] = n < 0 ? kGroupDefault[m][1] : n;
  }
  return prev;
}
