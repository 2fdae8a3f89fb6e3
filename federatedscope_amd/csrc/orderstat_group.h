// Internal to libfsagg: the K-wave form of the register radix select for
// 255 < n <= 512 clients — the coordinate-wise median
// (median_aggregator.py:43-52) and trimmed mean (trimmedmean_aggregator.py:
// 44-57).  Not part of the public ABI.
//
// A column of n > 255 values does not fit one lane's registers, and the
// one-lane streaming kernel (orderstat_stream.hip) reads it from HBM twice
// (histogram pass, compaction pass: FETCH 2.05 x 4nP).  Here the column's
// rows are split over the K = ceil(n / kGroupRows) waves of one workgroup
// (<= H values per lane per wave, 4 waves per SIMD at H <= 64), so the whole
// column is read ONCE and every pass runs from registers:
//  1. each wave loads its rows and takes |x|max of them; the K maxima meet
//     in LDS (barrier);
//  2. all waves add their values' octave digits (8 codes per octave, as the
//     register kernel) into one shared histogram of 16-bit counters — 256
//     bins in 128 LDS words per lane, [word][lane] — (barrier); wave 0 scans
//     it and hands both ranks' bins to the others through LDS (barrier);
//  3. refinement rounds (rare: while the two bins would overflow a wave's
//     list region) likewise;
//  4. compaction: wave w lists its bin values into its own region of the
//     lane's 256-word list area ([w·R, (w+1)·R), R = 256 / K; a miss lands
//     on the region's next free slot, the total listed count <= R − 1 bounds
//     every wave's), and sums its clamped middle terms (trimmed mean,
//     TrimBounds); each wave leaves its count and partial sum in LDS
//     (barrier) and all but wave 0 exit;
//  5. wave 0 reads the K regions as one list (positions mapped through the
//     counts' prefix), sorts it, reads the ranks off and writes the result.
// Algorithmic bytes per coordinate: 4·n read + 4 (base) + 4 written, in one
// pass.
#pragma once

#include "orderstat_pair.h"  // pair_rows, sel_put / sel_get

namespace fsagg {
namespace os {
namespace {

constexpr int kGroupRows = 64;   // rows per wave: H <= 64 fits 128 VGPRs
constexpr int kGroupMaxWaves = 8;     // n <= 512: larger n streams
constexpr int kGroupWords = 256;  // per-lane LDS words: histogram, then list
constexpr int kGroupHistWords = 128;

// 16-bit counter of bin d (d < 256): half d & 1 of word d / 2 ([word][lane]
// with a 256-B word stride: the word offset is (d >> 1) << 8)
__device__ __forceinline__ void hist16w_inc(uint32_t hb, uint32_t d) {
  __hip_atomic_fetch_add(lds_at(hb | ((d << 7) & 0x7F00u)),
                         1u << ((d & 1u) << 4), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Ranks ra, rb among the W words of 16-bit counters (2W bins): groups of
// four words (v_sad_u16 sums a word's halves into the running count), then
// the word, then the half.  Returns each rank's bin, the count below it and
// in it.
template <int W>
__device__ __forceinline__ void hist16w_find2(const uint32_t *H, int ra,
                                             int rb, uint32_t &da, int &ba,
                                             int &ca, uint32_t &db, int &bb,
                                             int &cb) {
  int cum = 0, na = 0, fa = 0, nb = 0, fb = 0;
#pragma unroll
  for (int q = 0; q < W / 4; ++q) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      cum = int(__builtin_amdgcn_sad_u16(H[(4 * q + i) * kWave], 0u,
                                         uint32_t(cum)));
    const bool ta = cum <= ra, tb = cum <= rb;
    na += ta;
    fa = ta ? cum : fa;
    nb += tb;
    fb = tb ? cum : fb;
  }
  auto in_group = [&](int g, int before, int r, int &below,
                      int &count) -> uint32_t {
    const uint32_t *G = H + 4 * g * kWave;
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = G[i * kWave];
    int c = before, k = 0, f = before;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      c = int(__builtin_amdgcn_sad_u16(x[i], 0u, uint32_t(c)));
      const bool t = c <= r;
      k += t;
      f = t ? c : f;
    }
    k = min(k, 3);
    uint32_t w = x[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) w = k == i ? x[i] : w;
    const int c0 = int(w & 0xFFFFu);
    const bool low = f + c0 > r;
    below = low ? f : f + c0;
    count = low ? c0 : int(w >> 16);
    return uint32_t(8 * g + 2 * k) + (low ? 0u : 1u);
  };
  da = in_group(min(na, W / 4 - 1), fa, ra, ba, ca);
  db = in_group(min(nb, W / 4 - 1), fb, rb, bb, cb);
}

// Refinement digit over 128 bins of 16-bit counters (cf. refine_plan): the
// bin's keys take digits <= 127, every key outside it the digit 128.
__device__ __forceinline__ Refine group_refine_plan(const RankSel &s) {
  Refine f;
  f.lo = s.lo;
  f.lim = s.hi - s.lo + 1u;
  int sh = max(0, 32 - __builtin_clz(f.lim | 1u) - 7);
  if (((f.lim + (1u << sh) - 1u) >> sh) > 127u) ++sh;
  f.sh = sh;
  f.pad = (0u - f.lim) & ((1u << sh) - 1u);
  return f;
}

// Wave 0's read of the K list regions as one list: position i lies in the
// region w whose counts' prefix p_w <= i < p_{w+1}, at slot w·R + i − p_w.
template <int S, bool SUM>
__device__ __forceinline__ void group_list_select(
    uint32_t hb, const int *pre, int K, int R, int cnt, int pa, int pb,
    int lo, int hi, uint32_t &va, uint32_t &vb, double &sum) {
  uint32_t a[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    int slot = i;  // region 0
#pragma unroll
    for (int w = 1; w < kGroupMaxWaves; ++w)
      slot = w < K && i >= pre[w] ? w * R + i - pre[w] : slot;
    const uint32_t x =
        ukey(*lds_at(hb | (uint32_t(slot & (kGroupWords - 1)) << 8)));
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

// 4 waves per SIMD: the VGPR budget is 128 (H values + the state)
template <int H, int MODE>
__global__ __launch_bounds__(kGroupMaxWaves * kWave)
__attribute__((amdgpu_waves_per_eu(4))) void orderstat_group_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  // histogram words [0, 128) then the K list regions over [0, 256); 64 KiB
  // aligned so a lane's word addresses are hb | (w << 8)
  __shared__ __attribute__((aligned(65536))) uint32_t lds[kGroupWords * kWave];
  __shared__ uint32_t xch[kGroupMaxWaves * kWave];   // maxima, then counts
  __shared__ uint32_t xmid[2 * kGroupMaxWaves * kWave];
  __shared__ uint32_t xsel[8 * kWave];
  const int K = int(blockDim.x) >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
  const int lane = int(threadIdx.x) & (kWave - 1);
  uint32_t *Hs = lds + lane;
  const uint32_t hb = uint32_t(uintptr_t((lds_u32 *)Hs));
  const BlockRows br = pair_rows(rs, blockIdx.x);
  if (br.len <= 0) return;  // a chunk's missing quarter (block-uniform)
  // wave w's rows [j0, j0 + nw): n split as evenly as K allows
  const int j0 = int((int64_t(n) * wv) / K);
  const int nw = int((int64_t(n) * (wv + 1)) / K) - j0;
  const float *const *__restrict__ rows = br.rows + j0;
  const float *__restrict__ base = br.base;
  const bool live = lane < br.len;
  __builtin_assume(nw >= H - 8 && nw <= H);  // dispatch
  const int R = kGroupWords / K;            // list region per wave
  const int cap = min(R - 1, 62);           // listed values the list takes
  // 1. this wave's rows; |x|max over all waves
  uint32_t u[H];
  float bval = 0.0f;
  {
    const uint32_t off = uint32_t(live ? br.lo + lane : br.lo);
#pragma unroll
    for (int j = 0; j < H; ++j)
      u[j] = __float_as_uint(ld_nt(row_at(rows, j < nw ? j : nw - 1), off));
    if (base && wv == 0) bval = ld_nt(base, off);
    xch[wv * kWave + lane] = abs_max_bits<H>(u);
  }
  // the histogram clear, shared out over the waves
  for (int w = wv; w < kGroupHistWords; w += K) Hs[w * kWave] = 0u;
  __syncthreads();
  uint32_t amax = 0u;
  for (int w = 0; w < K; ++w) amax = max(amax, xch[w * kWave + lane]);
  const bool nan = amax > 0x7F800000u;
  const bool nonfinite = amax >= 0x7F800000u;
  const uint32_t obase = octave_base(amax);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;

  // 2. the shared histogram; wave 0 finds both ranks' bins
  RankSel s1, s2;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    if (j >= H - 8 && j >= nw) continue;  // pads
    hist16w_inc(hb, octave_digit(u[j], obase));
  }
  __syncthreads();
  if (wv == 0) {
    uint32_t d1, d2;
    int b1, c1, b2, c2;
    hist16w_find2<kGroupHistWords>(Hs, r1, r2, d1, b1, c1, d2, b2, c2);
    octave_bin(d1, obase, s1.lo, s1.hi);
    octave_bin(d2, obase, s2.lo, s2.hi);
    s1.below = b1;
    s1.cnt = c1;
    s2.below = b2;
    s2.cnt = c2;
    sel_put(xsel, lane, s1, s2);
  }
  __syncthreads();
  if (wv != 0) sel_get(xsel, lane, s1, s2);

  // 3. refine while the two bins would overflow a region (rare)
  bool shared = same_bin(s1, s2);
#pragma unroll 1
  for (int round = 0; round < 12; ++round) {
    const bool list1 = !resolved(s1), list2 = !shared && !resolved(s2);
    const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
    const bool need = stored > cap;
    if (!__any(need)) break;
    const bool pick2 = list2 && (!list1 || s2.cnt > s1.cnt);
    fence_regs<H>(u);
    const Refine f = group_refine_plan(pick2 ? s2 : s1);
    for (int w = wv; w < 68; w += K) Hs[w * kWave] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < H; ++j) {
      if (j >= H - 8 && j >= nw) continue;
      const uint32_t rel = min(ukey(u[j]) - f.lo, f.lim);
      hist16w_inc(hb, (rel + f.pad) >> f.sh);
    }
    __syncthreads();
    if (wv == 0) {
      uint32_t da, db;
      int ba, ca, bb, cb;
      const int ra = pick2 ? r2 - s2.below : r1 - s1.below;
      hist16w_find2<68>(Hs, ra, r2 - s2.below, da, ba, ca, db, bb, cb);
      refine_apply(s2, f, need && shared, db, bb, cb);
      refine_apply(s2, f, need && pick2, da, ba, ca);
      refine_apply(s1, f, need && !pick2, da, ba, ca);
      sel_put(xsel, lane, s1, s2);
    }
    __syncthreads();
    if (wv != 0) sel_get(xsel, lane, s1, s2);
    shared = same_bin(s1, s2);
  }

  // 4. compaction into this wave's region
  const bool list1 = !resolved(s1);
  const bool list2 = !shared && !resolved(s2);
  const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
  double mid = 0.0;
  int c = 0;
  fence_regs<H>(u);
  const uint32_t start = hb | (uint32_t(wv * R) << 8);
  if (__any(list1 || list2) || MODE == kTrimmed) {
    if constexpr (MODE == kMedian) {
      // ranks r1, r1 + 1 are adjacent: one key band covers both lists
      const uint32_t lo = list1 ? s1.lo : s2.lo;
      const uint32_t w =
          (list1 || list2) ? (list2 ? s2.hi : s1.hi) - lo + 1u : 0u;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if (j >= H - 8 && j >= nw) continue;
        *lds_at(start + (uint32_t(c) << 8)) = u[j];  // a miss: overwritten
        c = add_below(c, ukey(u[j]) - lo, w);
      }
    } else {
      const TrimBounds tb = trim_bounds(s1, s2, shared, list1, list2, n);
      float g = 0.0f;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if (j >= H - 8 && j >= nw) continue;
        trim_step(u[j], tb, g, c, start + (uint32_t(c) << 8));
        if (j % kMidGroup == kMidGroup - 1) {
          mid += double(g);
          g = 0.0f;
        }
      }
      mid += double(g) - (wv == 0 ? tb.corr : 0.0);
    }
  }
  xch[wv * kWave + lane] = uint32_t(c);
  if (MODE == kTrimmed) {
    const uint64_t m = __double_as_longlong(mid);
    xmid[(2 * wv) * kWave + lane] = uint32_t(m);
    xmid[(2 * wv + 1) * kWave + lane] = uint32_t(m >> 32);
  }
  __syncthreads();
  if (wv != 0) return;
  int pre[kGroupMaxWaves];
  pre[0] = 0;
#pragma unroll
  for (int w = 1; w < kGroupMaxWaves; ++w)
    pre[w] = w < K ? pre[w - 1] + int(xch[(w - 1) * kWave + lane]) : 1 << 30;
  if (MODE == kTrimmed) {
    mid = 0.0;
    for (int w = 0; w < K; ++w)
      mid += __longlong_as_double(int64_t(
          uint64_t(xmid[(2 * w) * kWave + lane]) |
          (uint64_t(xmid[(2 * w + 1) * kWave + lane]) << 32)));
  }

  // 5. wave 0: the ranks (and the kept sum) off the sorted list
  constexpr bool SUM = MODE == kTrimmed;
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
    group_list_select<64, SUM>(hb, pre, K, R, stored, rr1, pb, lo, hi, va, vb,
                               lsum);
  else if (__any(stored > 16))
    group_list_select<32, SUM>(hb, pre, K, R, stored, rr1, pb, lo, hi, va, vb,
                               lsum);
  else if (__any(stored > 8))
    group_list_select<16, SUM>(hb, pre, K, R, stored, rr1, pb, lo, hi, va, vb,
                               lsum);
  else if (__any(stored > 0))
    group_list_select<8, SUM>(hb, pre, K, R, stored, rr1, pb, lo, hi, va, vb,
                              lsum);
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
