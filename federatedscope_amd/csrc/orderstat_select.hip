// Range-adaptive radix select with LDS compaction for the coordinate-wise
// median (median_aggregator.py:43-52) and trimmed mean
// (trimmedmean_aggregator.py:44-57), for SEL_N - kSelStep < n <= SEL_N.
// Compiled once per SEL_N (Makefile) so the register-heavy instantiations
// build in parallel.
//
// Keys stay in registers (one lane = one coordinate).  Per lane:
//  1. kmin/kmax of the column give the common key prefix; the first 8-bit
//     digit is the 8 bits just below it, so the first histogram splits the
//     column's actual value range (clustered deltas included), not the
//     sign/exponent byte.
//  2. One private 256-bin histogram of byte counters in LDS (ds_add_u32 of
//     1 << 8·(d & 3) into word d / 4; n <= 255 keeps every byte from
//     overflowing) places both needed ranks in their bins; one pass over its
//     64 words finds both.  While the keys of the two bins would overflow
//     the 64-slot list, the bins are refined by their next 7-bit digits,
//     both in one pass over the keys (rank 1's bins in histogram words
//     [0, 32), rank 2's in [32, 64)).
//  3. One compaction pass writes the keys of both bins to one per-lane LDS
//     list (bin 1 before bin 2 in key order, so the sorted list holds both
//     ranks) and, for the trimmed mean, sums every key strictly between the
//     bins in fp64.  The list is sorted in registers with the compile-time
//     bitonic network (32 or 64 keys) and the ranks read off.
// Histogram words and list slots are laid out [slot][lane], so the 64 lanes
// of a wave always hit 64 distinct banks.  The compaction stores every key
// at the list's current end (branch-free); a key outside both bins is
// overwritten by the next one inside, and word 64 catches the stores made
// once the list is full.
//
// Register budget: SEL_N keys + ~40 must stay within 256 VGPRs (2 waves per
// SIMD); SEL_N moves in steps of kSelStep so no more than 7 are padding.
#include "orderstat.h"

#ifndef SEL_N
#error "compile with -DSEL_N=<keys per lane>"
#endif

namespace fsagg {
namespace os {
namespace {

constexpr int kSelWords = 65;                    // 64 hist/list words + dump
constexpr int kSelWaves = kBlock / kWave;
constexpr int kSelLds = kSelWords * kWave * kSelWaves;  // 66.5 KiB per block
constexpr int kList = 64;  // LDS list slots per lane (slot 64: dump)
constexpr uint32_t kKeyPosInf = 0xFF800000u;  // f2key(+inf)
constexpr uint32_t kKeyNegInf = 0x007FFFFFu;  // f2key(-inf)

// Selection state of one rank.  Its bin is the keys whose bits >= lvl equal
// P's (P's lower bits are zero); `below` keys sort before the bin and `cnt`
// are in it.  lvl == 0: all 32 bits resolved, the bin is `cnt` copies of P.
struct RankSel {
  uint32_t P;
  int lvl, below, cnt;
};

__device__ __forceinline__ uint32_t bin_mask(int lvl) {
  return lvl >= 32 ? 0u : (0xFFFFFFFFu << lvl);
}
// shift of the next digit of `width` bits
__device__ __forceinline__ int digit_shift(const RankSel &s, int width = 8) {
  return s.lvl > width ? s.lvl - width : 0;
}

__device__ __forceinline__ RankSel rank_init(uint32_t kmin, uint32_t kmax,
                                             int n) {
  RankSel s;
  s.below = 0;
  s.cnt = n;
  s.lvl = kmin == kmax ? 0 : 32 - __builtin_clz(kmin ^ kmax);
  s.P = kmin & bin_mask(s.lvl);
  return s;
}

__device__ __forceinline__ void hist_clear(uint32_t *H) {
#pragma unroll
  for (int w = 0; w < 64; ++w) H[w * kWave] = 0u;
}

// Histogram address of digit d = (key >> sh) & 255: byte d & 3 of word d / 4.
// (v_bfe_u32 + v_lshl_add_u32 for the address; the shift amount of the
// value uses only its low 5 bits, so ((key >> sh) << 3) needs no mask.)
__device__ __forceinline__ uint32_t *hist_word(uint32_t *H, uint32_t key,
                                               int sh) {
  return H + __builtin_amdgcn_ubfe(key, uint32_t(sh + 2), 6u) * kWave;
}
__device__ __forceinline__ uint32_t hist_one(uint32_t key, int sh) {
  return 1u << (((key >> sh) << 3) & 31u);
}

// First digit: every real key of the lane (all share the common prefix).
template <int N>
__device__ __forceinline__ void hist_add_all(uint32_t *H,
                                             const uint32_t (&k)[N], int n,
                                             int sh) {
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j >= N - kSelStep && j >= n) continue;  // pads
    atomicAdd(hist_word(H, k[j], sh), hist_one(k[j], sh));
  }
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

template <bool TWO, int W = 64>
__device__ __forceinline__ void hist_scan(const uint32_t *H, int ra, int rb,
                                          uint32_t &da, int &ba, int &ca,
                                          uint32_t &db, int &bb, int &cb) {
  int ga, fa, gb, fb;
  group_find<TWO, W>(H, ra, rb, ga, fa, gb, fb);
  da = word_find(H, ga, fa, ra, ba, ca);
  if (TWO) db = word_find(H, gb, fb, rb, bb, cb);
}

// Refinement: the next 7-bit digit of the keys of BOTH ranks' bins in one
// pass — rank 1's bin counts into histogram words [0, 32), rank 2's into
// [32, 64) (the bins are disjoint unless shared, and then only rank 1's is
// counted); other keys and lanes add zeros.
template <int N>
__device__ __forceinline__ void hist_add_dual(uint32_t *H,
                                              const uint32_t (&k)[N], int n,
                                              const RankSel &s1, bool on1,
                                              const RankSel &s2, bool on2) {
  const int sh1 = digit_shift(s1, 7), sh2 = digit_shift(s2, 7);
  const uint32_t M1 = bin_mask(s1.lvl), M2 = bin_mask(s2.lvl);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j >= N - kSelStep && j >= n) continue;
    const uint32_t key = k[j];
    const bool m1 = on1 && (key & M1) == s1.P;
    const bool m2 = on2 && (key & M2) == s2.P;
    const uint32_t d = __builtin_amdgcn_ubfe(key, uint32_t(m2 ? sh2 : sh1),
                                             7u) | (m2 ? 128u : 0u);
    atomicAdd(&H[(d >> 2) * kWave],
              (m1 || m2) ? 1u << ((d & 3u) * 8u) : 0u);
  }
}

// Refinement of rank 1's bin alone (the common case: the median's two
// ranks share a bin): the key's offset from the bin base, shifted to the
// next 7-bit digit and clamped to 128, is the digit for keys in the bin; a
// key outside it lands in bin 128 (word 32, outside the 32-word scan) or,
// when the bin has fewer than 128 digits, in a digit above the bin's own —
// after every key of the bin, so the scan for a rank inside the bin never
// reaches it.  No compare/select per key.  (Lanes whose rank needs no
// refinement count garbage and ignore the result; <= 255 keys per lane
// keep every byte counter in range.)
template <int N>
__device__ __forceinline__ void hist_add_one(uint32_t *H,
                                             const uint32_t (&k)[N], int n,
                                             const RankSel &s) {
  const int sh = digit_shift(s, 7);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (j >= N - kSelStep && j >= n) continue;
    const uint32_t d = min((k[j] - s.P) >> sh, 128u);
    atomicAdd(&H[(d >> 2) * kWave], 1u << ((d << 3) & 31u));
  }
}

// Narrow s to digit bin d (count b below it, c in it), if on.
__device__ __forceinline__ void rank_apply(RankSel &s, bool on, uint32_t d,
                                           int b, int c, int width = 8) {
  if (!on) return;
  const int sh = digit_shift(s, width);
  s.below += b;
  s.cnt = c;
  s.P |= d << sh;
  s.lvl = sh;
}

__device__ __forceinline__ bool same_bin(const RankSel &a, const RankSel &b) {
  return a.lvl == b.lvl && a.P == b.P;
}

// Sort the lane's list of `cnt` keys at LDS slots [0, cnt) and read list
// positions pa and pb off it; Σ key2f over positions [lo, hi] in fp64.
template <int S, bool SUM>
__device__ __forceinline__ void list_select(const uint32_t *H, int cnt,
                                            int pa, int pb, int lo, int hi,
                                            uint32_t &va, uint32_t &vb,
                                            double &sum) {
  uint32_t a[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const uint32_t x = H[i * kWave];
    a[i] = i < cnt ? x : kPad;
  }
  bitonic_sort<S>(a);
  uint32_t xa = 0, xb = 0;
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    xa = i == pa ? a[i] : xa;
    xb = i == pb ? a[i] : xb;
    if (SUM) acc += (i >= lo && i <= hi) ? double(key2f(a[i])) : 0.0;
  }
  va = xa;
  vb = xb;
  sum = acc;
}

template <int N, int MODE>
__global__ __launch_bounds__(kBlock) void orderstat_select_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  __shared__ uint32_t lds[kSelLds];
  uint32_t *H = lds + (threadIdx.x / kWave) * kSelWords * kWave +
                (threadIdx.x & (kWave - 1));
  const BlockRows br = block_rows(rs, blockIdx.x);
  const float *const *__restrict__ rows = br.rows;
  const float *__restrict__ base = br.base;
  const int64_t p = br.lo + threadIdx.x;
  const bool live = int(threadIdx.x) < br.len;
  __builtin_assume(n > N - kSelStep && n <= N);  // dispatch
  uint32_t k[N];
  {
    // coordinates < 2^30 (launch); dead lanes re-read the chunk's first
    const uint32_t off = uint32_t(live ? p : br.lo);
#pragma unroll
    for (int j = 0; j < N; ++j)
      k[j] = __float_as_uint(ld_nt(rows[j < n ? j : n - 1], off));
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const uint32_t key = f2key(__uint_as_float(k[j]));
      k[j] = (j < N - kSelStep || j < n) ? key : kPad;
    }
  }
  bool nan, nonfinite;
  RankSel s1;
  {
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j >= N - kSelStep && j >= n) continue;
      kmin = min(kmin, k[j]);
      kmax = max(kmax, k[j]);
    }
    nan = kmax > kKeyPosInf || kmin < kKeyNegInf;
    nonfinite = kmax >= kKeyPosInf || kmin <= kKeyNegInf;
    s1 = rank_init(kmin, kmax, n);
  }
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;
  // first digit: one histogram places both ranks
  RankSel s2 = s1;
  if (__any(s1.lvl > 0)) {
    const bool on = s1.lvl > 0;
    hist_clear(H);
    hist_add_all<N>(H, k, n, digit_shift(s1));
    uint32_t d1, d2;
    int b1, c1, b2, c2;
    hist_scan<true>(H, r1, r2, d1, b1, c1, d2, b2, c2);
    rank_apply(s1, on, d1, b1, c1);
    rank_apply(s2, on, d2, b2, c2);
  }
  // The keys of both rank bins go to one LDS list of at most kList keys
  // (bin 1 then bin 2 in key order).  Refine a bin with more than
  // kList / 2 keys while the list would overflow.
  bool shared = same_bin(s1, s2);
#pragma unroll 1
  for (int round = 0; round < 4; ++round) {  // 7-bit digits: lvl 24 → 0
    const bool list1 = s1.lvl > 0, list2 = !shared && s2.lvl > 0;
    const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
    const bool need1 =
        list1 && stored > kList && (shared || s1.cnt > kList / 2);
    const bool need2 = list2 && stored > kList && s2.cnt > kList / 2;
    if (!__any(need1 || need2)) break;
    hist_clear(H);
    if (__any(need2))
      hist_add_dual<N>(H, k, n, s1, need1, s2, need2);
    else
      hist_add_one<N>(H, k, n, s1);
    uint32_t d1, d2, d3 = 0;
    int b1, c1, b2, c2, b3 = 0, c3 = 0;
    // rank 1 (and rank 2 where it shares rank 1's bin) in words [0, 32)
    hist_scan<true, 32>(H, r1 - s1.below, r2 - s2.below, d1, b1, c1, d2, b2,
                        c2);
    // rank 2 in its own bin: words [32, 64)
    if (__any(need2))
      hist_scan<false, 32>(H + 32 * kWave, r2 - s2.below, 0, d3, b3, c3, d3,
                           b3, c3);
    rank_apply(s2, need1 && shared, d2, b2, c2, 7);
    rank_apply(s2, need2, d3, b3, c3, 7);
    rank_apply(s1, need1, d1, b1, c1, 7);
    shared = same_bin(s1, s2);
  }

  // compaction: the keys of the listed bins, in row order
  const bool list1 = s1.lvl > 0;
  const bool list2 = !shared && s2.lvl > 0;
  const uint32_t lo1 = s1.P, hi1 = s1.P | ~bin_mask(s1.lvl);
  const uint32_t lo2 = s2.P, hi2 = s2.P | ~bin_mask(s2.lvl);
  double mid = 0.0;
  // (no per-key test of "any list" — that compiles to a branch per key; a
  // lane with no list writes slots nobody reads: stored == 0 below)
  if (__any(list1 || list2) || MODE == kTrimmed) {
    int c = 0;
    if constexpr (MODE == kMedian) {
      // ranks r1, r1 + 1 are adjacent: no key lies between the two bins, so
      // one key range covers both lists
      const uint32_t lo = list1 ? lo1 : lo2;
      const uint32_t span = (list2 ? hi2 : hi1) - lo;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j >= N - kSelStep && j >= n) continue;
        const uint32_t key = k[j];
        const bool m = key - lo <= span;
        H[min(c, kList) * kWave] = key;  // a miss: overwritten by next hit
        c += m;
      }
    } else {
      const uint32_t span1 = list1 ? hi1 - lo1 : 0u;
      const uint32_t l1 = list1 ? lo1 : 0xFFFFFFFFu;
      const uint32_t span2 = list2 ? hi2 - lo2 : 0u;
      const uint32_t l2 = list2 ? lo2 : 0xFFFFFFFFu;
      // strictly between the bins: (hi1, lo2)
      const uint32_t mlo = hi1 + 1u;
      const uint32_t mspan = shared ? 0u : lo2 - mlo;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        if (j >= N - kSelStep && j >= n) continue;
        const uint32_t key = k[j];
        const bool m = key - l1 <= span1 || key - l2 <= span2;
        // select in fp32, then widen: one v_cndmask, not a 64-bit pair
        const float x = key - mlo < mspan ? key2f(key) : 0.0f;
        mid += double(x);
        H[min(c, kList) * kWave] = key;  // a miss: overwritten by next hit
        c += m;
      }
    }
  }

  // read the ranks (and the kept sum) off the sorted list
  constexpr bool SUM = MODE == kTrimmed;
  const int rr1 = r1 - s1.below, rr2 = r2 - s2.below;
  const int c1off = list1 ? s1.cnt : 0;
  const int stored = c1off + (list2 ? s2.cnt : 0);
  const int pb = shared ? rr2 : c1off + rr2;
  int lo, hi;
  double fixed = 0.0;  // kept copies of fully resolved (unlisted) bins
  if (shared) {
    lo = list1 ? rr1 : 0;
    hi = list1 ? rr2 : -1;
    if (!list1) fixed = double(key2f(s1.P)) * double(rr2 - rr1 + 1);
  } else {
    lo = list1 ? rr1 : 0;
    hi = list2 ? c1off + rr2 : c1off - 1;
    if (!list1) fixed += double(key2f(s1.P)) * double(s1.cnt - rr1);
    if (!list2) fixed += double(key2f(s2.P)) * double(rr2 + 1);
  }
  uint32_t va = 0, vb = 0;
  double lsum = 0.0;
  // the smallest network that holds every lane's list
  if (__any(stored > 32))
    list_select<kList, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 16))
    list_select<32, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 8))
    list_select<16, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  else if (__any(stored > 0))
    list_select<8, SUM>(H, stored, rr1, pb, lo, hi, va, vb, lsum);
  const uint32_t v1 = list1 ? va : s1.P;
  const uint32_t v2 = (shared ? list1 : list2) ? vb : s2.P;
  const double sum1 = lsum + fixed, sum2 = 0.0;
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
    float s = float(sum1 + mid + sum2);
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
  if (base) r = add_rn(gld(base + p), r);
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
