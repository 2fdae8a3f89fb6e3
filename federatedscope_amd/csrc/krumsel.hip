// Krum's certified selection on the device, straight from the Gram chain's
// finish buffer, and the selected clients' average tables
// (fsagg_krum_select_f32; include/fsagg.h).
//
// The host certificate (csrc/host/krumcert.cpp, restating
// core/aggregators/_engine.ambiguous_clients) needs the n x n finish buffer
// on the host: one device-to-host round trip after the chain, then the
// certificate, the subset's row table and weights, their upload and the
// average's launch — ~70 us of host latency between the last Gram kernel and
// the average at C4 (tools/time_krum_phases.py).  Here two small kernels do
// the same on the device right behind the chain, and write the selected
// clients' row table, weights and base table for the row-set weighted sum
// (fsagg_weighted_sum_rows_f32), which the caller launches behind them; the
// host reads back one flag and the order and only falls back to its own
// path when the selection is not certified.
//
// Scores (krum_aggregator.py:75-77): the sum of each row's k = n − f − 2
// smallest distances, over D64 (the fp64 key sums), and the interval
// [lo, hi] over max(D64 − B64, 0) and D64 + B64 (B64 = max(B, Bᵀ) +
// (nseg + 2)·2^-52·D64), scaled by (1 ∓ 1e-12) — exactly the host's
// quantities; only the order in which each row's k values are added differs
// (a tree here, nth_element order there), which moves a sum by roundings
// far inside the 1e-12 slack.  The order is the stable sort of the scores;
// the certificate is krumcert.cpp's: unordered, the chosen m's largest hi
// below the rest's smallest lo; ordered (multi-Krum's average sums the
// chosen in score order), every position i < m clearing every later client.
#include <cmath>
#include <cstdint>

#include "common.h"

namespace fsagg {
namespace {

constexpr int kSelBlock = 256;
static_assert(FSAGG_KRUMSEL_MAX_CLIENTS <= kSelBlock,
              "one thread per client");

struct KrumArgs {
  double size[FSAGG_KRUMSEL_MAX_CLIENTS];       // sample sizes (weights)
  const float *base[FSAGG_KRUMSEL_MAX_SEGS];    // init model, per key
};

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// grid n: block a, thread b < n — row a's three k-smallest sums
// (work[0..n) scores, [n, 2n) lo, [2n, 3n) hi) and its flags (work[3n + a])
__global__ __launch_bounds__(kSelBlock) void krum_scores_kernel(
    const int32_t *__restrict__ buf, int n, int nseg, int k,
    double *__restrict__ work) {
  __shared__ double v[3][kSelBlock];
  __shared__ double part[3][kSelBlock / kWave];
  __shared__ uint32_t fl;
  const int a = blockIdx.x, b = threadIdx.x;
  const size_t nn = size_t(n) * n;
  const double *D64 = reinterpret_cast<const double *>(buf);
  const uint32_t *flag = reinterpret_cast<const uint32_t *>(buf) + 3 * nn;
  const float *B = reinterpret_cast<const float *>(buf) + 4 * nn;
  const double form = double(nseg + 2) * 0x1p-52;
  if (b == 0) fl = 0u;
  __syncthreads();
  if (b < n) {
    const double d = D64[size_t(a) * n + b];
    double bnd = fmax(double(B[size_t(a) * n + b]), double(B[size_t(b) * n + a]));
    bnd += form * (isfinite(d) ? d : 0.0);
    v[0][b] = d;
    v[1][b] = fmax(d - bnd, 0.0);
    v[2][b] = d + bnd;
    if (flag[size_t(a) * n + b] != 0u) atomicOr(&fl, 1u);
  }
  __syncthreads();
  double s[3] = {0.0, 0.0, 0.0};
  if (b < n) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double x = v[j][b];
      int r = 0;
      for (int c = 0; c < n; ++c) {
        const double y = v[j][c];
        r += (y < x || (y == x && c < b)) ? 1 : 0;
      }
      if (r < k) s[j] = x;
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    s[j] = wave_sum(s[j]);
    if ((b & (kWave - 1)) == 0) part[j][b / kWave] = s[j];
  }
  __syncthreads();
  if (b == 0) {
    double t[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      t[j] = 0.0;
      for (int w = 0; w < kSelBlock / kWave; ++w) t[j] += part[j][w];
    }
    work[a] = t[0];
    work[n + a] = t[1] * (1.0 - 1e-12);
    work[2 * n + a] = t[2] * (1.0 + 1e-12);
    work[3 * n + a] = fl ? 1.0 : 0.0;
  }
}

// one block: the stable order, the certificate, and the first msel clients'
// row table [nsegt][msel] (from tab [nsegt][n], ss = n, or [1][n], ss = 0),
// fp32 weights and base table.  sel[0] = 1 when certified, sel[1] = 1 when
// the scores are usable at all (no flagged pair, k > 0), sel[2 + i] =
// order[i].
__global__ __launch_bounds__(kSelBlock) void krum_pick_kernel(
    const double *__restrict__ work, int n, int k, int m, int ordered,
    const KrumArgs args, int wmode, int nseg, const int64_t *__restrict__ tab,
    int64_t ss, int nsegt, int32_t *__restrict__ sel,
    int64_t *__restrict__ sub_tab, float *__restrict__ sub_w,
    int64_t *__restrict__ sub_base) {
  __shared__ double sc[kSelBlock], lo[kSelBlock], hi[kSelBlock];
  __shared__ double suf[kSelBlock + 1];
  __shared__ int o[kSelBlock];
  __shared__ int bad;
  __shared__ double total;
  const int a = threadIdx.x;
  if (a == 0) bad = 0;
  __syncthreads();
  if (a < n) {
    sc[a] = work[a];
    lo[a] = work[n + a];
    hi[a] = work[2 * n + a];
    if (work[3 * n + a] != 0.0 || !isfinite(work[a])) atomicOr(&bad, 1);
  }
  __syncthreads();
  if (a < n) {
    const double x = sc[a];
    int pos = 0;
    for (int b = 0; b < n; ++b) {
      const double y = sc[b];
      pos += (y < x || (y == x && b < a)) ? 1 : 0;
    }
    o[pos] = a;
  }
  __syncthreads();
  const int msel = m < n ? m : n;
  if (a == 0) {
    const bool valid = bad == 0 && k > 0;
    bool amb = false;
    if (valid && m > 0) {
      int mm = m;
      bool check = true;
      if (m >= n) {
        if (!ordered) check = false;
        mm = n - 1;
      }
      if (check) {
        suf[n] = __builtin_inf();
        for (int i = n - 1; i >= 0; --i) suf[i] = fmin(suf[i + 1], lo[o[i]]);
        if (!ordered) {
          double top = -__builtin_inf();
          for (int i = 0; i < mm; ++i) top = fmax(top, hi[o[i]]);
          amb = !(top < suf[mm]);
        } else {
          for (int i = 0; i < mm && !amb; ++i) amb = hi[o[i]] >= suf[i + 1];
        }
      }
    }
    sel[0] = valid && !amb ? 1 : 0;
    sel[1] = valid ? 1 : 0;
    double t = 0.0;
    for (int i = 0; i < msel; ++i) t += args.size[o[i]];
    total = t;
  }
  __syncthreads();
  if (a < n) sel[2 + a] = o[a];
  if (a < msel) {
    const int c = o[a];
    for (int s = 0; s < nsegt; ++s)
      sub_tab[int64_t(s) * msel + a] = tab[int64_t(s) * ss + c];
    // fedavg_weights (core/aggregators/_engine.py): size / total in fp64
    // (Python's int / int is correctly rounded, and so is this division of
    // the exactly represented doubles), 1/m with ignore_weight; rounded to
    // fp32 as the kernels' weights are
    const double w = wmode == 1 ? 1.0 / double(msel) : args.size[c] / total;
    sub_w[a] = float(w);
  }
  if (a < nseg && sub_base) sub_base[a] = int64_t(uintptr_t(args.base[a]));
}

}  // namespace
}  // namespace fsagg

extern "C" int fsagg_krum_select_f32(
    const int32_t *buf, int n, int nseg, int f, int m, int ordered,
    const double *sizes, int ignore_weight, const float *const *base,
    const int64_t *tab, int64_t ss, int nsegt, double *work, int32_t *sel,
    int64_t *sub_tab, float *sub_w, int64_t *sub_base,
    fsagg_stream_t stream) {
  using namespace fsagg;
  if (!buf || n < 1 || n > FSAGG_KRUMSEL_MAX_CLIENTS || nseg < 1 || m < 1 ||
      !sizes || !tab || (ss != 0 && ss != n) || nsegt < 1 ||
      (ss == 0 && nsegt != 1) || !work || !sel || !sub_tab || !sub_w ||
      (base && (nseg > FSAGG_KRUMSEL_MAX_SEGS || !sub_base))) {
    set_error("fsagg_krum_select_f32: invalid argument (n=%d nseg=%d m=%d "
              "ss=%lld nsegt=%d)", n, nseg, m, (long long)ss, nsegt);
    return FSAGG_EINVAL;
  }
  KrumArgs args;
  for (int i = 0; i < FSAGG_KRUMSEL_MAX_CLIENTS; ++i)
    args.size[i] = i < n ? sizes[i] : 0.0;
  for (int s = 0; s < FSAGG_KRUMSEL_MAX_SEGS; ++s)
    args.base[s] = base && s < nseg ? base[s] : nullptr;
  hipStream_t st = as_stream(stream);
  const int k = n - f - 2;
  hipLaunchKernelGGL(krum_scores_kernel, dim3(n), dim3(kSelBlock), 0, st, buf,
                     n, nseg, k, work);
  hipLaunchKernelGGL(krum_pick_kernel, dim3(1), dim3(kSelBlock), 0, st, work,
                     n, k, m, ordered, args, ignore_weight ? 1 : 0,
                     base ? nseg : 0, tab, ss, nsegt, sel, sub_tab, sub_w,
                     base ? sub_base : nullptr);
  return check_launch("fsagg_krum_select_f32");
}
