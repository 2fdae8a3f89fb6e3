// Octave-digit radix select with LDS compaction for the coordinate-wise
// median (median_aggregator.py:43-52) and trimmed mean
// (trimmedmean_aggregator.py:44-57), for SEL_N - kSelStep < n <= SEL_N.
// Compiled once per SEL_N (Makefile) so the register-heavy instantiations
// build in parallel.
//
// One lane owns one coordinate; its n values stay in registers as raw float
// bits (so the trimmed mean's middle sum needs no key-to-float decode).
//  1. Load pass: the column's largest magnitude |x|max (one and + half a
//     max3 per value) — it also flags NaN/inf.
//  2. One histogram of an *octave digit* places both needed ranks: a value's
//     magnitude code m = 8 exponent bits + 3 mantissa bits (8 codes per
//     octave) relative to |x|max's code, clamped to the 128 codes (16
//     octaves) below it, on the value's sign side — digits 0..127 negative
//     (large magnitudes first), 128..255 positive.  Monotone in the value,
//     so each rank's digit is a key interval.  Unlike a digit of raw key
//     bits, whose top byte spans two octaves per bin, the octave digit splits
//     the bulk of a column finely whatever its signs: at C5 (N(0,1) with 10 %
//     ×100 outliers) the rank bins hold ~2-10 values where the top byte's
//     held ~50.  Byte counters, 256 bins in 64 words of LDS per lane
//     ([word][lane], 64 distinct banks per wave).
//  3. If the two rank bins hold more than the 64-slot list, the larger bin is
//     refined by a linear digit of its key interval (the fallback for columns
//     spanning more than 16 octaves, e.g. exact zeros or huge outliers);
//     every round shrinks a bin ≥ 2^6-fold, so 10 rounds always suffice.
//  4. One compaction pass writes the keys of both bins to one per-lane LDS
//     list (bin 1 before bin 2 in key order) and, for the trimmed mean, sums
//     every value strictly between the bins in fp64.  The list is sorted with
//     the smallest sorting network that holds every lane's list and the ranks
//     (and the kept partial sums) read off.
// Register budget: SEL_N values + ~40 within 256 VGPRs (2 waves per SIMD).
#include "orderstat_sel.h"
#include "orderstat_pair.h"

#ifndef SEL_N
#error "compile with -DSEL_N=<keys per lane>"
#endif

namespace fsagg {
namespace os {
namespace {

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_select_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  // 16 KiB-aligned: a lane's word addresses are hb | (w << 8)
  __shared__ __attribute__((aligned(16384))) uint32_t lds[kSelLds];
  uint32_t *H = lds + (threadIdx.x / kWave) * kSelWords * kWave +
                (threadIdx.x & (kWave - 1));
  const uint32_t hb = uint32_t(uintptr_t((lds_u32 *)H));
  const BlockRows br = block_rows(rs, blockIdx.x);
  const float *const *__restrict__ rows = br.rows;
  const float *__restrict__ base = br.base;
  const int64_t p = br.lo + threadIdx.x;
  const bool live = int(threadIdx.x) < br.len;
  __builtin_assume(n > N - kSelStep && n <= N);  // dispatch
  // 1. the column as raw float bits; |x|max.  Rows past n (pads) re-read
  // row n - 1: harmless for the max, skipped by every counting pass.
  uint32_t u[N];
  uint32_t amax = 0u;
  float bval = 0.0f;  // the init model's coordinate (init + update)
  {
    // coordinates < 2^30 (launch); dead lanes re-read the chunk's first
    const uint32_t off = uint32_t(live ? p : br.lo);
#pragma unroll
    for (int j = 0; j < N; ++j)
      u[j] = __float_as_uint(ld_nt(row_at(rows, j < n ? j : n - 1), off));
    // with the rows, not at the end: a load issued as the wave's last act
    // exposes one full HBM round trip per wave (0.14 ms at C5)
    if (base) bval = ld_nt(base, off);
    amax = abs_max_bits<N>(u);
  }
  const bool nan = amax > 0x7F800000u;
  const bool nonfinite = amax >= 0x7F800000u;
  const uint32_t obase = octave_base(amax);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;

  // 2. octave-digit histogram: both ranks' bins
  RankSel s1, s2;
  {
    hist_clear(H, 64);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j >= N - kSelStep && j >= n) continue;  // pads
      hist_inc(hb, octave_digit(u[j], obase));
    }
    uint32_t d1, d2;
    int b1, c1, b2, c2;
    hist_scan<true, 64>(H, r1, r2, d1, b1, c1, d2, b2, c2);
    octave_bin(d1, obase, s1.lo, s1.hi);
    octave_bin(d2, obase, s2.lo, s2.hi);
    s1.below = b1;
    s1.cnt = c1;
    s2.below = b2;
    s2.cnt = c2;
  }

  // 3. refine while the two bins would overflow the list (rare)
  bool shared = same_bin(s1, s2);
#pragma unroll 1
  for (int round = 0; round < 10; ++round) {
    const bool list1 = !resolved(s1), list2 = !shared && !resolved(s2);
    const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
    const bool need = stored > kList;
    if (!__any(need)) break;
    // the larger listed bin (a shared bin carries both ranks)
    const bool pick2 = list2 && (!list1 || s2.cnt > s1.cnt);
    fence_regs<N>(u);
    const Refine f = refine_plan(pick2 ? s2 : s1);
    hist_clear(H, 33);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j >= N - kSelStep && j >= n) continue;
      const uint32_t rel = min(ukey(u[j]) - f.lo, f.lim);
      hist_inc(hb, (rel + f.pad) >> f.sh);
    }
    uint32_t da, db;
    int ba, ca, bb, cb;
    const int ra = pick2 ? r2 - s2.below : r1 - s1.below;
    hist_scan<true, 32>(H, ra, r2 - s2.below, da, ba, ca, db, bb, cb);
    refine_apply(s2, f, need && shared, db, bb, cb);
    refine_apply(s2, f, need && pick2, da, ba, ca);
    refine_apply(s1, f, need && !pick2, da, ba, ca);
    shared = same_bin(s1, s2);
  }

  // 4. compaction: the values of the listed bins, in row order (at most
  // kList, so the running slot c never passes the dump slot kList)
  const bool list1 = !resolved(s1);
  const bool list2 = !shared && !resolved(s2);
  double mid = 0.0;
  fence_regs<N>(u);
  if (__any(list1 || list2) || MODE == kTrimmed) {
    int c = 0;
    if constexpr (MODE == kMedian) {
      // ranks r1, r1 + 1 are adjacent: no key lies between the two bins, so
      // one key range [lo, lo + w) covers both lists.  When it lies on one
      // side of zero (every lane of the wave), it is one interval of the
      // float bits themselves, [ulo, ulo + w): no key transform per value.
      const uint32_t lo = list1 ? s1.lo : s2.lo;
      const uint32_t w =
          (list1 || list2) ? (list2 ? s2.hi : s1.hi) - lo + 1u : 0u;
      const uint32_t hi = lo + (w - 1u);
      const bool pos = lo >= 0x80000000u, neg = hi < 0x80000000u;
      if (!__any(w != 0u && !pos && !neg)) {
        const uint32_t ulo = pos ? lo - 0x80000000u : ~hi;
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (j >= N - kSelStep && j >= n) continue;
          *lds_at(hb | (uint32_t(c) << 8)) = u[j];  // a miss: overwritten
          c = add_below(c, u[j] - ulo, w);
        }
      } else {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          if (j >= N - kSelStep && j >= n) continue;
          *lds_at(hb | (uint32_t(c) << 8)) = u[j];  // a miss: overwritten
          c = add_below(c, ukey(u[j]) - lo, w);
        }
      }
    } else {
      // the listed bins as raw-bit intervals, the middle as Σ med3(x, L, U)
      // in fp32 groups of kMidGroup (orderstat_sel.h TrimBounds)
      const TrimBounds tb = trim_bounds(s1, s2, shared, list1, list2, n);
      float g = 0.0f;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j >= N - kSelStep && j >= n) continue;
        trim_step(u[j], tb, g, c, hb | (uint32_t(c) << 8));
        if (j % kMidGroup == kMidGroup - 1) {
          mid += double(g);
          g = 0.0f;
        }
      }
      mid += double(g) - tb.corr;
    }
  }

  // 5. read the ranks (and the kept sum) off the sorted list
  constexpr bool SUM = MODE == kTrimmed;
  const int rr1 = r1 - s1.below, rr2 = r2 - s2.below;
  const int c1off = list1 ? s1.cnt : 0;
  const int stored = c1off + (list2 ? s2.cnt : 0);
  const int pb = shared ? rr2 : c1off + rr2;
  int lo, hi;
  double fixed = 0.0;  // kept copies of resolved (unlisted) bins
  if (shared) {
    lo = list1 ? rr1 : 0;
    hi = list1 ? rr2 : -1;
    if (!list1) fixed = double(key2f(s1.lo)) * double(rr2 - rr1 + 1);
  } else {
    lo = list1 ? rr1 : 0;
    hi = list2 ? c1off + rr2 : c1off - 1;
    if (!list1) fixed += double(key2f(s1.lo)) * double(s1.cnt - rr1);
    if (!list2) fixed += double(key2f(s2.lo)) * double(rr2 + 1);
  }
  uint32_t va = 0, vb = 0;
  double lsum = 0.0;
  // the smallest network that holds every lane's list
  if (__any(stored > 32))
    list_select<64, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 16))
    list_select<32, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 8))
    list_select<16, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 0))
    list_select<8, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  const uint32_t v1 = list1 ? va : s1.lo;
  const uint32_t v2 = (shared ? list1 : list2) ? vb : s2.lo;
  if (!live) return;
  float r;
  if constexpr (MODE == kMedian) {
    // (median(T) - median(-T)) / 2, literally
    r = __fdiv_rn(key2f(v1) - (-key2f(v2)), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    // Σall − Σtop − Σbottom in fp32: with k >= 1 an infinity is always
    // among the excluded values, so inf - inf (or a NaN) gives NaN; with
    // k == 0 it is Σall itself, summed in row order (rare: re-read).
    float s = float(lsum + fixed + mid);
    if (nonfinite) {
      s = __builtin_nanf("");
      if (kk == 0 && !nan) {
        s = 0.0f;
#pragma unroll 1
        for (int j = 0; j < n; ++j) s = add_rn(s, gld(rows[j] + p));
      }
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(bval, r);
  out[p] = r;
}

}  // namespace

template <int N, int MODE>
void launch_select(const RowSrc &rs, unsigned grid, int n, int kk,
                   float divisor, float *out, hipStream_t s) {
  hipLaunchKernelGGL((orderstat_select_kernel<N, MODE>), dim3(grid),
                     dim3(kBlock), 0, s, rs, n, kk, divisor, out);
}

template void launch_select<SEL_N, kMedian>(const RowSrc &, unsigned, int,
                                            int, float, float *,
                                            hipStream_t);
template void launch_select<SEL_N, kTrimmed>(const RowSrc &, unsigned, int,
                                             int, float, float *,
                                             hipStream_t);

// the two-wave form (orderstat_pair.h): H = SEL_N / 2 values per wave
template <int H, int MODE>
void launch_pair(const RowSrc &rs, unsigned grid, int n, int kk,
                 float divisor, float *out, hipStream_t s) {
  hipLaunchKernelGGL((orderstat_pair_kernel<H, MODE>), dim3(grid),
                     dim3(kPairBlock), 0, s, rs, n, kk, divisor, out);
}

template void launch_pair<SEL_N / 2, kMedian>(const RowSrc &, unsigned, int,
                                              int, float, float *,
                                              hipStream_t);
template void launch_pair<SEL_N / 2, kTrimmed>(const RowSrc &, unsigned, int,
                                               int, float, float *,
                                               hipStream_t);

}  // namespace os
}  // namespace fsagg
