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
//     the smallest bitonic network that holds every lane's list and the ranks
//     (and the kept partial sums) read off.
// Register budget: SEL_N values + ~40 within 256 VGPRs (2 waves per SIMD).
#include "orderstat.h"

#ifndef SEL_N
#error "compile with -DSEL_N=<keys per lane>"
#endif

namespace fsagg {
namespace os {
namespace {

constexpr int kSelWords = 64;  // hist/list words per lane (list: 63 + dump)
constexpr int kSelWaves = kBlock / kWave;
constexpr int kSelLds = kSelWords * kWave * kSelWaves;  // 64 KiB per block
constexpr int kList = 63;      // LDS list slots per lane (slot 63: dump)
constexpr int kMagShift = 20;  // magnitude code: bits [30:20] of |x|
constexpr int kCodes = 128;    // codes per sign side (16 octaves)
constexpr uint32_t kKeyPosInf = 0xFF800000u;  // ukey(+inf)
constexpr uint32_t kKeyNegInf = 0x007FFFFFu;  // ukey(-inf)

// float bits -> order-preserving key (-0 < +0), 3 ops
__device__ __forceinline__ uint32_t ukey(uint32_t u) {
  return u ^ (uint32_t(int32_t(u) >> 31) | 0x80000000u);
}

// Selection state of one rank: its bin is the key interval [lo, hi] holding
// `cnt` keys, `below` keys sort before it.  lo == hi: resolved (cnt copies).
struct RankSel {
  uint32_t lo, hi;
  int below, cnt;
};

// c + (a < b): the borrow of a − b carried straight into the counter
// (v_sub_co_u32 + v_addc_co_u32, a VCC carry chain with no wait states).
// The compiler's own form is v_cmp + s_nop 1 + v_cndmask_b32_e64 + v_add —
// the wait states guard the e64 cndmask's read of VCC — one per value.
__device__ __forceinline__ int add_below(int c, uint32_t a, uint32_t b) {
  uint32_t t;
  asm("v_sub_co_u32 %1, vcc, %2, %3\n\t"
      "v_addc_co_u32 %0, vcc, 0, %0, vcc"
      : "+v"(c), "=&v"(t)
      : "v"(a), "v"(b)
      : "vcc");
  return c;
}

// Opaque copy barrier: keeps the compiler from hoisting per-pass key math
// (ukey of every value) out of a pass and holding N more registers live.
template <int N>
__device__ __forceinline__ void fence_regs(uint32_t (&u)[N]) {
#pragma unroll
  for (int j = 0; j < N; ++j) asm volatile("" : "+v"(u[j]));
}

__device__ __forceinline__ bool resolved(const RankSel &s) {
  return s.lo == s.hi;
}
__device__ __forceinline__ bool same_bin(const RankSel &a, const RankSel &b) {
  return a.lo == b.lo && a.hi == b.hi;
}

// Octave digit of float bits u (monotone in the value):
//   t = clamp(m(u) - base, 0, 127); digit = negative ? 127 - t : 128 + t
// ((t ^ sign) + 128 with sign = -1 or 0: v_xad_u32).
__device__ __forceinline__ uint32_t octave_digit(uint32_t u, int base) {
  const int m = int(__builtin_amdgcn_ubfe(u, uint32_t(kMagShift), 11u));
  const int t = min(max(m - base, 0), kCodes - 1);
  return (uint32_t(t) ^ uint32_t(int32_t(u) >> 31)) + 128u;
}

// The key interval of octave digit d (given the launch's base).
__device__ __forceinline__ void octave_bin(uint32_t d, int base, uint32_t &lo,
                                           uint32_t &hi) {
  const bool pos = d >= 128u;
  const int t = pos ? int(d) - 128 : 127 - int(d);
  const int mlo = t == 0 ? 0 : base + t;
  const int mhi = t == kCodes - 1 ? 2047 : base + t;
  // |x| bits [mlo << 20, (mhi << 20) | 0xFFFFF] (a selected bin is never
  // empty, so 0 <= mlo <= mhi)
  const uint32_t alo = uint32_t(max(mlo, 0)) << kMagShift;
  const uint32_t ahi = (uint32_t(max(mhi, 0)) << kMagShift) | 0xFFFFFu;
  // the top bins stop at ±inf, so no band [lo1, hi2] spans all 2^32 keys
  // (NaN keys lie outside every bin; a NaN column's result is NaN anyway)
  if (pos) {
    lo = alo | 0x80000000u;
    hi = min(ahi | 0x80000000u, kKeyPosInf);
  } else {
    lo = max(~(ahi | 0x80000000u), kKeyNegInf);
    hi = ~(alo | 0x80000000u);
  }
}

__device__ __forceinline__ void hist_clear(uint32_t *H, int words) {
#pragma unroll
  for (int w = 0; w < 64; ++w)
    if (w < words) H[w * kWave] = 0u;
}

// The lane's LDS words by byte address: word w at hb | (w << 8) ([word][lane]
// layout: a wave's 64 lanes hit 64 distinct banks).  hb = wave·16 KiB +
// lane·4 has bits 8..13 clear (the LDS array is 16 KiB-aligned), so a word
// address is one v_and_or / v_lshl_or.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ lds_u32 *lds_at(uint32_t byte) {
  return (lds_u32 *)(uintptr_t)byte;
}

// byte counter of digit d: byte d & 3 of word d / 4
__device__ __forceinline__ void hist_inc(uint32_t hb, uint32_t d) {
  __hip_atomic_fetch_add(lds_at(hb | ((d << 6) & 0x3F00u)),
                         1u << ((d << 3) & 31u), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Locate rank r in the histogram given the word that holds it (w, x) and
// the count before that word: returns the bin, the count below and in it.
__device__ __forceinline__ uint32_t hist_bin(int w, uint32_t x, int before,
                                            int r, int &below, int &count) {
  uint32_t byte = 3;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int c = int((x >> (8 * b)) & 255u);
    const bool stop = byte == 3 && before + c > r;
    byte = stop ? uint32_t(b) : byte;
    before += (byte == 3) ? c : 0;
  }
  below = before;
  count = int((x >> (8 * byte)) & 255u);
  return uint32_t(w) * 4u + byte;
}

// Rank ra (and rb if TWO) in W histogram words (from H), in two levels:
// the W / 4 groups of four words first (the word byte sums chained through
// v_sad_u8's accumulator), then the four words of the group holding the
// rank.  At either level the number of entries whose inclusive prefix count
// is <= r is the one holding r, and the last such prefix is the count
// before it.
template <bool TWO, int W>
__device__ __forceinline__ void group_find(const uint32_t *H, int ra, int rb,
                                           int &ga, int &fa, int &gb,
                                           int &fb) {
  int cum = 0, na = 0, ba = 0, nb = 0, bb = 0;
#pragma unroll
  for (int q = 0; q < W / 4; ++q) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      cum = int(__builtin_amdgcn_sad_u8(H[(4 * q + i) * kWave], 0u,
                                        uint32_t(cum)));
    const bool ta = cum <= ra;
    na += ta;
    ba = ta ? cum : ba;
    if (TWO) {
      const bool tb = cum <= rb;
      nb += tb;
      bb = tb ? cum : bb;
    }
  }
  ga = min(na, W / 4 - 1);
  fa = ba;
  gb = min(nb, W / 4 - 1);
  fb = bb;
}

__device__ __forceinline__ uint32_t word_find(const uint32_t *H, int g,
                                              int before, int r, int &below,
                                              int &count) {
  const uint32_t *G = H + 4 * g * kWave;
  uint32_t x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = G[i * kWave];
  int cum = before, n = 0, f = before;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cum = int(__builtin_amdgcn_sad_u8(x[i], 0u, uint32_t(cum)));
    const bool t = cum <= r;
    n += t;
    f = t ? cum : f;
  }
  n = min(n, 3);
  uint32_t w = x[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) w = n == i ? x[i] : w;
  return hist_bin(4 * g + n, w, f, r, below, count);
}

template <bool TWO, int W>
__device__ __forceinline__ void hist_scan(const uint32_t *H, int ra, int rb,
                                          uint32_t &da, int &ba, int &ca,
                                          uint32_t &db, int &bb, int &cb) {
  int ga, fa, gb, fb;
  group_find<TWO, W>(H, ra, rb, ga, fa, gb, fb);
  da = word_find(H, ga, fa, ra, ba, ca);
  if (TWO) db = word_find(H, gb, fb, rb, bb, cb);
}

// Linear refinement digit of a key interval [lo, lo + lim - 1]: rel =
// min(key - lo, lim) (keys below lo wrap, so every key outside maps to lim),
// digit = (rel + pad) >> sh with pad making lim + pad a multiple of 2^sh —
// the bin's keys take digits [pad >> sh, (lim - 1 + pad) >> sh] <= 127 and
// every key outside the bin the single digit above them (<= 128, word 32),
// which a scan for a rank inside the bin never reaches.
struct Refine {
  uint32_t lo, lim, pad;
  int sh;
};

__device__ __forceinline__ Refine refine_plan(const RankSel &s) {
  Refine f;
  f.lo = s.lo;
  f.lim = s.hi - s.lo + 1u;  // <= 2^31: a bin never crosses the sign
  int sh = max(0, 32 - __builtin_clz(f.lim | 1u) - 7);
  if (((f.lim + (1u << sh) - 1u) >> sh) > 127u) ++sh;
  f.sh = sh;
  f.pad = (0u - f.lim) & ((1u << sh) - 1u);
  return f;
}

// Narrow s to refinement digit d (count b below it, c in it).
__device__ __forceinline__ void refine_apply(RankSel &s, const Refine &f,
                                             bool on, uint32_t d, int b,
                                             int c) {
  if (!on) return;
  const uint32_t span = f.lim - 1u;
  const uint32_t r0 = d << f.sh;
  const uint32_t rlo = r0 > f.pad ? r0 - f.pad : 0u;
  const uint32_t r1 = ((d + 1u) << f.sh) - 1u - f.pad;
  const uint32_t rhi = r1 < span ? r1 : span;
  s.below += b;
  s.cnt = c;
  s.hi = f.lo + rhi;
  s.lo = f.lo + rlo;
}

// a[idx] for a per-lane idx without dynamic register indexing: a binary
// select tree, one lane mask per bit of idx (S − 1 v_cndmask and log2 S
// compares, where comparing idx with every position costs S of each plus a
// wait state per position)
template <int S>
__device__ __forceinline__ uint32_t tree_pick(const uint32_t (&a)[S],
                                              int idx) {
  uint32_t t[S];
#pragma unroll
  for (int i = 0; i < S; ++i) t[i] = a[i];
#pragma unroll
  for (int w = S / 2, b = 0; w >= 1; w /= 2, ++b) {
    const bool up = (idx >> b) & 1;
#pragma unroll
    for (int k = 0; k < w; ++k) t[k] = up ? t[2 * k + 1] : t[2 * k];
  }
  return t[0];
}

// Sort the lane's list of `cnt` values (float bits) at LDS slots [0, cnt) by
// key and read list positions pa and pb off it (as keys); Σ over positions
// [lo, hi] in fp64.
template <int S, bool SUM>
__device__ __forceinline__ void list_select(const uint32_t *H, int cnt,
                                            int pa, int pb, int lo, int hi,
                                            uint32_t &va, uint32_t &vb,
                                            double &sum) {
  uint32_t a[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint32_t x = ukey(H[i * kWave]);
    a[i] = i < cnt ? x : kPad;
  }
  bitonic_sort<S>(a);
  double acc = 0.0;
  if (SUM) {
    // [lo, hi] as one unsigned range test; an empty range (hi < lo) moves
    // lo far above every position so that no i passes
    const bool empty = hi < lo;
    const int lo1 = empty ? (1 << 30) : lo;
    const uint32_t span = empty ? 0u : uint32_t(hi - lo);
#pragma unroll
    for (int i = 0; i < S; ++i) {
      // select in fp32, then widen (one v_cndmask, not a 64-bit pair)
      float x = uint32_t(i - lo1) <= span ? key2f(a[i]) : 0.0f;
      asm("" : "+v"(x));
      acc += double(x);
    }
  }
  va = tree_pick<S>(a, pa);
  vb = tree_pick<S>(a, pb);
  sum = acc;
}

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
#pragma unroll
    for (int j = 0; j < N; ++j) amax = max(amax, u[j] & 0x7FFFFFFFu);
  }
  const bool nan = amax > 0x7F800000u;
  const bool nonfinite = amax >= 0x7F800000u;
  const int obase = int(amax >> kMagShift) - (kCodes - 1);
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
      // the band from bin 1 to bin 2 relative to A: [0, w1) bin 1 listed,
      // [w1, w1 + wm) strictly between the bins (summed), then bin 2 listed
      // up to wb
      const uint32_t A = list1 ? s1.lo : s1.hi + 1u;
      const uint32_t w1 = list1 ? s1.hi - s1.lo + 1u : 0u;
      const uint32_t wm = shared ? 0u : s2.lo - (s1.hi + 1u);
      const uint32_t wb = w1 + wm + (list2 ? s2.hi - s2.lo + 1u : 0u);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j >= N - kSelStep && j >= n) continue;
        const uint32_t rel = ukey(u[j]) - A;
        const bool inm = rel - w1 < wm;
        // select in fp32, then widen: one v_cndmask, not a 64-bit pair (the
        // empty asm keeps the compiler from sinking the select past the cvt)
        float x = inm ? __uint_as_float(u[j]) : 0.0f;
        asm("" : "+v"(x));
        mid += double(x);
        *lds_at(hb | (uint32_t(c) << 8)) = u[j];  // a miss: overwritten
        c += (rel < wb) && !inm;
      }
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

}  // namespace os
}  // namespace fsagg
