// Internal to libfsagg: the two-wave form of the register radix select
// (orderstat_select.hip), for the coordinate-wise median
// (median_aggregator.py:43-52) and trimmed mean (trimmedmean_aggregator.py:
// 44-57).  Not part of the public ABI.
//
// Why two waves per column.  The one-wave kernel holds a lane's whole column
// in registers: n = 200 values + ~45 VGPRs leaves 2 waves per SIMD.  gfx950
// issues a wave's VALU instructions at most every ~5 cycles, two waves'
// together every ~2.6 (profiles/r03/valu_issue_probe.txt), so whenever one
// wave of the pair is loading, the other computes at half the SIMD's rate —
// and at C5 a wave's 5.3k VALU instructions take longer than its 200 loads.
// Here the column's rows are split between two waves of one workgroup (wave
// 0 rows [0, ⌈n/2⌉), wave 1 the rest): H = ⌈n/2⌉ values per lane, 3 waves
// per SIMD at n = 200 (4 at n <= 128), and the per-value VALU work is spread
// over more resident waves, so a loading wave leaves two others to issue.
//
// The waves share one histogram (byte counters: at most n <= 255 per bin)
// and one per-lane list in LDS, both indexed by lane (the same 64
// coordinates in both waves):
//  1. each wave loads its rows and takes |x|max of them; the two maxima meet
//     in LDS (barrier);
//  2. both waves add their values' octave digits into the shared histogram
//     (barrier); wave 0 scans it and hands both ranks' bins to wave 1
//     through LDS (barrier), so every later wave-level decision (refinement
//     rounds, network size) agrees;
//  3. refinement rounds (rare) likewise;
//  4. compaction: wave 0 lists its bin values from slot 0 up, wave 1 from
//     slot kPairTop = 62 down (slots [0, 62]); each wave's misses land
//     on its next free slot, which lies in the gap between the two fills
//     (stored <= 62), so no valid entry is ever overwritten.  Trimmed mean:
//     each wave sums its strictly-middle values; wave 1 leaves its partial
//     and exits;
//  5. wave 0 reads the list (the top fill remapped), sorts it with the
//     smallest network holding every lane's list, reads the ranks off and
//     writes the result.
// Algorithmic bytes per coordinate: 4·n read + 4 (base) + 4 written.
#pragma once

#include "orderstat_sel.h"

namespace fsagg {
namespace os {
namespace {

constexpr int kPairBlock = 2 * kWave;
constexpr int kPairList = 62;  // list slots [0, 62); slot 62 a shared dump
constexpr int kPairTop = 62;   // wave 1's fill starts at slot 62 (down)

// Block b's 64 coordinates: flat form [64·b, ...); row-set form, quarter
// b & 3 of chunk b >> 2 (chunks hold <= kBlock = 4·64 coordinates).
__device__ __forceinline__ BlockRows pair_rows(const RowSrc &rs, int b) {
  BlockRows br;
  int seg = 0;
  if (rs.chunks) {
    const int sub = (b & 3) * kWave;
    br.lo = rs.chunks[b >> 2].lo + sub;
    br.len = rs.chunks[b >> 2].len - sub;
    seg = rs.chunks[b >> 2].seg;
  } else {
    br.lo = int64_t(b) * kWave;
    const int64_t r = rs.numel - br.lo;
    br.len = r < kWave ? int(r) : kWave;
  }
  br.rows = rs.tab + int64_t(seg) * rs.ss;
  br.base = rs.btab ? rs.btab[int64_t(seg) * rs.bss] : rs.base;
  return br;
}

// The LDS byte address of list slot `start + dir·c` for this lane: one
// v_mad_i32_i24 (step = ±256 bytes, the word stride of the [word][lane]
// layout), so both waves run the same compaction loop — wave 0 filling up
// from slot 0, wave 1 down from slot kPairTop.
__device__ __forceinline__ uint32_t slot_addr(int c, int step, uint32_t base) {
  uint32_t a;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(a) : "v"(c), "s"(step), "v"(base));
  return a;
}

// Wave 0's list read: positions [0, c0) are slots [0, c0) (its own fill),
// positions [c0, cnt) are wave 1's fill read from slot kPairTop down.
template <int S, bool SUM>
__device__ __forceinline__ void pair_list_select(uint32_t hb, int c0, int cnt,
                                                 int pa, int pb, int lo,
                                                 int hi, uint32_t &va,
                                                 uint32_t &vb, double &sum) {
  uint32_t a[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int slot = i < c0 ? i : kPairTop + c0 - i;
    const uint32_t x = ukey(*lds_at(hb | (uint32_t(slot & 63) << 8)));
    a[i] = i < cnt ? x : kPad;
  }
  sort_network<S>(a);
  double acc = 0.0;
  if (SUM) {
    const bool empty = hi < lo;
    const int lo1 = empty ? (1 << 30) : lo;
    const uint32_t span = empty ? 0u : uint32_t(hi - lo);
#pragma unroll
    for (int i = 0; i < S; ++i) {
      float x = uint32_t(i - lo1) <= span ? key2f(a[i]) : 0.0f;
      asm("" : "+v"(x));
      acc += double(x);
    }
  }
  va = tree_pick<S>(a, pa);
  vb = tree_pick<S>(a, pb);
  sum = acc;
}

template <int H, int MODE>
__device__ __forceinline__ void pair_compact(const uint32_t (&u)[H], int nw,
                                             int n, bool first,
                                             uint32_t start, int step,
                                             const RankSel &s1,
                                             const RankSel &s2, bool shared,
                                             bool list1, bool list2, int &c,
                                             double &mid) {
  c = 0;
  if constexpr (MODE == kMedian) {
    const uint32_t lo = list1 ? s1.lo : s2.lo;
    const uint32_t w =
        (list1 || list2) ? (list2 ? s2.hi : s1.hi) - lo + 1u : 0u;
    const uint32_t hi = lo + (w - 1u);
    const bool pos = lo >= 0x80000000u, neg = hi < 0x80000000u;
    if (!__any(w != 0u && !pos && !neg)) {
      const uint32_t ulo = pos ? lo - 0x80000000u : ~hi;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if (j >= H - 4 && j >= nw) continue;
        *lds_at(slot_addr(c, step, start)) = u[j];  // a miss: overwritten
        c = add_below(c, u[j] - ulo, w);
      }
    } else {
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if (j >= H - 4 && j >= nw) continue;
        *lds_at(slot_addr(c, step, start)) = u[j];
        c = add_below(c, ukey(u[j]) - lo, w);
      }
    }
  } else {
    // the trimmed mean's bins and middle (orderstat_sel.h TrimBounds); the
    // correction of the clamped sum is taken once, by wave 0
    const TrimBounds tb = trim_bounds(s1, s2, shared, list1, list2, n);
    float g = 0.0f;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      if (j >= H - 4 && j >= nw) continue;
      trim_step(u[j], tb, g, c, slot_addr(c, step, start));
      if (j % kMidGroup == kMidGroup - 1) {
        mid += double(g);
        g = 0.0f;
      }
    }
    mid += double(g) - (first ? tb.corr : 0.0);
  }
}

// Wave 0 scans the shared histogram and hands both ranks' bins to wave 1
// through LDS (8 words per lane) instead of both waves scanning it.
__device__ __forceinline__ void sel_put(uint32_t *X, int lane, const RankSel &a,
                                        const RankSel &b) {
  X[0 * kWave + lane] = a.lo;
  X[1 * kWave + lane] = a.hi;
  X[2 * kWave + lane] = uint32_t(a.below);
  X[3 * kWave + lane] = uint32_t(a.cnt);
  X[4 * kWave + lane] = b.lo;
  X[5 * kWave + lane] = b.hi;
  X[6 * kWave + lane] = uint32_t(b.below);
  X[7 * kWave + lane] = uint32_t(b.cnt);
}

__device__ __forceinline__ void sel_get(const uint32_t *X, int lane,
                                        RankSel &a, RankSel &b) {
  a.lo = X[0 * kWave + lane];
  a.hi = X[1 * kWave + lane];
  a.below = int(X[2 * kWave + lane]);
  a.cnt = int(X[3 * kWave + lane]);
  b.lo = X[4 * kWave + lane];
  b.hi = X[5 * kWave + lane];
  b.below = int(X[6 * kWave + lane]);
  b.cnt = int(X[7 * kWave + lane]);
}

template <int H, int MODE>
__global__ __launch_bounds__(kPairBlock) void orderstat_pair_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  // one histogram / list of 64 words per coordinate, shared by both waves;
  // 16 KiB-aligned so a lane's word addresses are hb | (w << 8)
  __shared__ __attribute__((aligned(16384))) uint32_t lds[kSelWords * kWave];
  __shared__ uint32_t xch[2 * kWave];
  __shared__ uint32_t xsel[8 * kWave];
  const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
  const int lane = int(threadIdx.x) & (kWave - 1);
  uint32_t *Hs = lds + lane;
  const uint32_t hb = uint32_t(uintptr_t((lds_u32 *)Hs));
  const BlockRows br = pair_rows(rs, blockIdx.x);
  if (br.len <= 0) return;  // a chunk's missing quarter (block-uniform)
  const int n0 = (n + 1) >> 1;
  const int nw = wv ? n - n0 : n0;
  const float *const *__restrict__ rows = br.rows + (wv ? n0 : 0);
  const float *__restrict__ base = br.base;
  const bool live = lane < br.len;
  __builtin_assume(nw > H - 5 && nw <= H);  // dispatch: 2H - 8 < n <= 2H
  // 1. this wave's rows as raw float bits; |x|max over both waves
  uint32_t u[H];
  uint32_t amax = 0u;
  float bval = 0.0f;
  {
    const uint32_t off = uint32_t(live ? br.lo + lane : br.lo);
#pragma unroll
    for (int j = 0; j < H; ++j)
      u[j] = __float_as_uint(ld_nt(row_at(rows, j < nw ? j : nw - 1), off));
    if (base && wv == 0) bval = ld_nt(base, off);
    amax = abs_max_bits<H>(u);
  }
  xch[wv * kWave + lane] = amax;
  // the histogram clear, half per wave
#pragma unroll
  for (int w = 0; w < 32; ++w) Hs[(wv * 32 + w) * kWave] = 0u;
  __syncthreads();
  amax = max(xch[lane], xch[kWave + lane]);
  const bool nan = amax > 0x7F800000u;
  const bool nonfinite = amax >= 0x7F800000u;
  const uint32_t obase = octave_base(amax);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;

  // 2. the shared octave-digit histogram: both ranks' bins, found by wave 0
  RankSel s1, s2;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    if (j >= H - 4 && j >= nw) continue;  // pads
    hist_inc(hb, octave_digit(u[j], obase));
  }
  __syncthreads();
  if (wv == 0) {
    uint32_t d1, d2;
    int b1, c1, b2, c2;
    hist_scan<true, 64>(Hs, r1, r2, d1, b1, c1, d2, b2, c2);
    octave_bin(d1, obase, s1.lo, s1.hi);
    octave_bin(d2, obase, s2.lo, s2.hi);
    s1.below = b1;
    s1.cnt = c1;
    s2.below = b2;
    s2.cnt = c2;
    sel_put(xsel, lane, s1, s2);
  }
  // after this barrier wave 0 is done reading the histogram (the list may
  // overwrite it) and wave 1 holds the same bins
  __syncthreads();
  if (wv == 1) sel_get(xsel, lane, s1, s2);

  // 3. refine while the two bins would overflow the list (rare); both waves
  // hold the same bins, so they take the same number of rounds
  bool shared = same_bin(s1, s2);
#pragma unroll 1
  for (int round = 0; round < 10; ++round) {
    const bool list1 = !resolved(s1), list2 = !shared && !resolved(s2);
    const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
    const bool need = stored > kPairList;
    if (!__any(need)) break;
    const bool pick2 = list2 && (!list1 || s2.cnt > s1.cnt);
    fence_regs<H>(u);
    const Refine f = refine_plan(pick2 ? s2 : s1);
#pragma unroll
    for (int w = 0; w < 17; ++w)
      if (wv * 17 + w < 33) Hs[(wv * 17 + w) * kWave] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < H; ++j) {
      if (j >= H - 4 && j >= nw) continue;
      const uint32_t rel = min(ukey(u[j]) - f.lo, f.lim);
      hist_inc(hb, (rel + f.pad) >> f.sh);
    }
    __syncthreads();
    if (wv == 0) {
      uint32_t da, db;
      int ba, ca, bb, cb;
      const int ra = pick2 ? r2 - s2.below : r1 - s1.below;
      hist_scan<true, 32>(Hs, ra, r2 - s2.below, da, ba, ca, db, bb, cb);
      refine_apply(s2, f, need && shared, db, bb, cb);
      refine_apply(s2, f, need && pick2, da, ba, ca);
      refine_apply(s1, f, need && !pick2, da, ba, ca);
      sel_put(xsel, lane, s1, s2);
    }
    __syncthreads();
    if (wv == 1) sel_get(xsel, lane, s1, s2);
    shared = same_bin(s1, s2);
  }

  // 4. compaction into the shared list, wave 0 from the bottom, wave 1 from
  // the top (after both waves have read the histogram for the last time)
  const bool list1 = !resolved(s1);
  const bool list2 = !shared && !resolved(s2);
  const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
  double mid = 0.0;
  int c = 0;
  fence_regs<H>(u);
  if (__any(list1 || list2) || MODE == kTrimmed)
    pair_compact<H, MODE>(u, nw, n, wv == 0,
                          wv ? hb | (kPairTop << 8) : hb,
                          wv ? -256 : 256, s1, s2, shared, list1, list2, c,
                          mid);
  if (MODE == kTrimmed && wv == 1) {
    const uint64_t m = __double_as_longlong(mid);
    xch[lane] = uint32_t(m);
    xch[kWave + lane] = uint32_t(m >> 32);
  }
  __syncthreads();
  if (wv == 1) return;
  if (MODE == kTrimmed)
    mid += __longlong_as_double(int64_t(uint64_t(xch[lane]) |
                                        (uint64_t(xch[kWave + lane]) << 32)));

  // 5. wave 0: read the ranks (and the kept sum) off the sorted list
  constexpr bool SUM = MODE == kTrimmed;
  const int c0 = c;
  const int rr1 = r1 - s1.below, rr2 = r2 - s2.below;
  const int c1off = list1 ? s1.cnt : 0;
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
  if (__any(stored > 32))
    pair_list_select<64, SUM>(hb, c0, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 16))
    pair_list_select<32, SUM>(hb, c0, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 8))
    pair_list_select<16, SUM>(hb, c0, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 0))
    pair_list_select<8, SUM>(hb, c0, stored, rr1, pb, lo, hi, va, vb, lsum);
  const uint32_t v1 = list1 ? va : s1.lo;
  const uint32_t v2 = (shared ? list1 : list2) ? vb : s2.lo;
  if (!live) return;
  const int64_t p = br.lo + lane;
  float r;
  if constexpr (MODE == kMedian) {
    r = __fdiv_rn(key2f(v1) - (-key2f(v2)), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
    float s = float(lsum + fixed + mid);
    if (nonfinite) {
      s = __builtin_nanf("");
      if (kk == 0 && !nan) {
        s = 0.0f;
#pragma unroll 1
        for (int j = 0; j < n; ++j) s = add_rn(s, gld(br.rows[j] + p));
      }
    }
    r = __fdiv_rn(s, divisor);
  }
  if (base) r = add_rn(bval, r);
  out[p] = r;
}

}  // namespace
}  // namespace os
}  // namespace fsagg
