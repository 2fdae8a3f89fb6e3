// Internal to libfsagg: device helpers of the radix-select order-statistic
// kernels — the register form (orderstat_select.hip, 32 < n <= 56 and
// 64 < n <= 255) and the streaming form (orderstat_stream.hip, n > 255).
// Not part of the public ABI.
#pragma once

#include "orderstat.h"

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

// |x|max of a lane's values as float bits (NaN flagged: > 0x7F800000), from
// a signed and an unsigned max chain (v_max3_i32 / v_max3_u32: one op per
// value in all, against an and + half a max3 for max(u & 0x7FFFFFFF)): the
// signed max is the largest non-negative value's bits, the unsigned max the
// largest negative one's magnitude with the sign bit on top.
template <int N>
__device__ __forceinline__ uint32_t abs_max_bits(const uint32_t (&u)[N]) {
  int32_t smax = int32_t(0x80000000u);
  uint32_t umax = 0u;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    smax = max(smax, int32_t(u[j]));
    umax = max(umax, u[j]);
  }
  const uint32_t pos = smax >= 0 ? uint32_t(smax) : 0u;
  const uint32_t neg = umax >= 0x80000000u ? umax & 0x7FFFFFFFu : 0u;
  return max(pos, neg);
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

// Octave digit of float bits u (monotone in the value), base >= 0:
//   t = max(m(u) - base, 0); digit = negative ? 127 - t : 128 + t
// (t <= 127 because m(u) <= the column's largest code, which the launch
// puts at most 127 above base; one saturating v_sub_u32 for the clamp;
// (t ^ sign) + 128 with sign = -1 or 0: v_xad_u32).
__device__ __forceinline__ uint32_t octave_digit(uint32_t u, uint32_t base) {
  const uint32_t m = __builtin_amdgcn_ubfe(u, uint32_t(kMagShift), 11u);
  const uint32_t t = __builtin_elementwise_sub_sat(m, base);
  return (t ^ uint32_t(int32_t(u) >> 31)) + 128u;
}

// The digit base of a column whose largest magnitude bits are amax: its
// code 127 digits up, clamped at 0 (a column of tiny values then uses the
// codes from 0: still monotone, octave_bin takes the same base).
__device__ __forceinline__ uint32_t octave_base(uint32_t amax) {
  return uint32_t(max(int(amax >> kMagShift) - (kCodes - 1), 0));
}

// The key interval of octave digit d (given the launch's base).
__device__ __forceinline__ void octave_bin(uint32_t d, uint32_t ubase,
                                           uint32_t &lo, uint32_t &hi) {
  const int base = int(ubase);
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

// The trimmed mean's compaction bounds.  Each listed bin as an
// interval of RAW float bits [lo, lo + w) — a bin never holds both signs, and
// positive keys k are the bits k − 2^31, negative ones ~k (order reversed) —
// so membership is one subtract and one borrow, no key transform per value
// (w = 0: the bin is not listed).  The values strictly between the bins are
// summed as Σ med3(x, L, U) over every value, L = the largest value of bin 1
// and U = the smallest of bin 2: a value at or below L adds L, one at or
// above U adds U, so Σmiddle = Σmed3 − L·#(key <= bin 1) − U·#(key >= bin 2),
// the counts known from the histogram (corr below; exact in fp64).  ±0 may
// land on either side of a zero bound, where it adds 0 either way.
// The clamped middle terms are summed in fp32 over groups of kMidGroup
// values, each group widened into the fp64 total: a group of m terms is off
// by at most (m − 1)·u·Σ|terms| (u = 2^-24; m <= 12 where pad rows fold into
// the last group), inside the reference's own fp32 cascade bound.
constexpr int kMidGroup = 8;

struct TrimBounds {
  uint32_t lo1, w1, lo2, w2;
  float L, U;
  double corr;
};

__device__ __forceinline__ void raw_bin(const RankSel &s, bool listed,
                                        uint32_t &lo, uint32_t &w) {
  w = listed ? s.hi - s.lo + 1u : 0u;
  lo = s.lo >= 0x80000000u ? s.lo - 0x80000000u : ~s.hi;
}

__device__ __forceinline__ TrimBounds trim_bounds(const RankSel &s1,
                                                  const RankSel &s2,
                                                  bool shared, bool list1,
                                                  bool list2, int n) {
  TrimBounds b;
  raw_bin(s1, list1, b.lo1, b.w1);
  raw_bin(s2, list2, b.lo2, b.w2);
  if (shared) {  // both ranks in one bin: no middle
    b.L = b.U = 0.0f;
    b.corr = 0.0;
  } else {
    b.L = key2f(s1.hi);
    b.U = key2f(s2.lo);
    b.corr = double(b.L) * double(s1.below + s1.cnt) +
             double(b.U) * double(n - s2.below);
  }
  return b;
}

// One value of the trimmed compaction: its clamped middle term into the
// fp32 group sum g, its bits into list slot c (a miss is overwritten by the
// next value), c advanced when it lies in a listed bin.
__device__ __forceinline__ void trim_step(uint32_t u, const TrimBounds &b,
                                          float &g, int &c, uint32_t addr) {
  g = add_rn(g, __builtin_amdgcn_fmed3f(__uint_as_float(u), b.L, b.U));
  // in place: left to itself the compiler sinks the med3s and adds to the
  // end of the pass and holds every value's term live
  asm volatile("" : "+v"(g));
  *lds_at(addr) = u;
  c = add_below(c, u - b.lo1, b.w1);
  c = add_below(c, u - b.lo2, b.w2);
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
  sort_network<S>(a);
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

}  // namespace
}  // namespace os
}  // namespace fsagg
