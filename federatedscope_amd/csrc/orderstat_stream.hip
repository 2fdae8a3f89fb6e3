// Coordinate-wise median (median_aggregator.py:43-52) and trimmed mean
// (trimmedmean_aggregator.py:44-57) for n > 255 clients: the octave-digit
// radix select of orderstat_select.hip with the column streamed from memory
// in every pass instead of held in registers.
//
// One lane owns one coordinate.  A column of n > 255 values no longer fits a
// lane's registers, and the register kernel's byte counters would overflow,
// so each pass re-reads the column (coalesced: one 256-B row segment per
// wave-instruction, 32 rows in flight per lane; plain loads, so the later
// passes hit the caches where the workgroup's rows are still resident):
//  1. the largest finite |x| of the first 64 rows (the digit's base: any
//     base gives exact bins, the sample only sets how finely they split the
//     bulk) and the init coordinate;
//  2. a histogram of a 128-bin octave digit (4 codes per octave, 16 octaves
//     below the base, per sign side) in 16-bit LDS counters — the same 64
//     LDS words per lane as the register kernel's 256 byte counters —
//     places both ranks (and flags NaN/inf);
//  3. while the two rank bins would overflow the 63-slot list, the larger
//     is refined by a 64-bin linear digit of its key interval (every round
//     shrinks it 64-fold; rare);
//  4. one compaction pass lists both bins' values (and, for the trimmed
//     mean, sums every value strictly between them in fp64); the list is
//     sorted and the ranks read off, as in the register kernel.
// Two column reads (and 64 rows) in the common case, against the 2·32 of
// the bit-by-bit select it replaces (orderstat.hip
// orderstat_generic_kernel, kept for n > 65535).  Algorithmic bytes per coordinate: 4·n + 4 read, 4 written.
#include <cstdlib>

#include "orderstat_sel.h"


namespace fsagg {
namespace os {
namespace {

constexpr int kStMagShift = 21;  // magnitude code: bits [30:21] of |x|
constexpr int kStCodes = 64;     // codes per sign side (16 octaves)
constexpr int kStRefineBins = 64;
constexpr int kStSample = 64;    // rows that set the digit's base

__device__ __forceinline__ uint32_t st_digit(uint32_t u, int base) {
  const int m = int(__builtin_amdgcn_ubfe(u, uint32_t(kStMagShift), 10u));
  const int t = min(max(m - base, 0), kStCodes - 1);
  return (uint32_t(t) ^ uint32_t(int32_t(u) >> 31)) + uint32_t(kStCodes);
}

// key interval of digit d (cf. octave_bin)
__device__ __forceinline__ void st_bin(uint32_t d, int base, uint32_t &lo,
                                       uint32_t &hi) {
  const bool pos = d >= uint32_t(kStCodes);
  const int t = pos ? int(d) - kStCodes : kStCodes - 1 - int(d);
  const int mlo = t == 0 ? 0 : base + t;
  const int mhi = t == kStCodes - 1 ? 1023 : base + t;
  const uint32_t alo = uint32_t(max(mlo, 0)) << kStMagShift;
  const uint32_t ahi =
      (uint32_t(max(mhi, 0)) << kStMagShift) | ((1u << kStMagShift) - 1u);
  if (pos) {
    lo = alo | 0x80000000u;
    hi = min(ahi | 0x80000000u, kKeyPosInf);
  } else {
    lo = max(~(ahi | 0x80000000u), kKeyNegInf);
    hi = ~(alo | 0x80000000u);
  }
}

// 16-bit counter of bin d (d < 128): half d & 1 of word d / 2
__device__ __forceinline__ void hist16_inc(uint32_t hb, uint32_t d) {
  __hip_atomic_fetch_add(lds_at(hb | ((d << 7) & 0x3F00u)),
                         1u << ((d & 1u) << 4), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Rank r among 128 16-bit counters: groups of four words (8 bins) first
// (v_sad_u16 sums a word's halves into the running count), then the word,
// then the half.  Returns the bin; `below` = count before it, `count` in it.
__device__ __forceinline__ void hist16_find2(const uint32_t *H, int ra,
                                            int rb, uint32_t &da, int &ba,
                                            int &ca, uint32_t &db, int &bb,
                                            int &cb) {
  int cum = 0, na = 0, fa = 0, nb = 0, fb = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
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
  da = in_group(min(na, 15), fa, ra, ba, ca);
  db = in_group(min(nb, 15), fb, rb, bb, cb);
}

// 64-bin refinement digit of a key interval (cf. refine_plan): in-bin keys
// take digits <= 63, every key outside the single digit 64
__device__ __forceinline__ Refine st_refine_plan(const RankSel &s) {
  Refine f;
  f.lo = s.lo;
  f.lim = s.hi - s.lo + 1u;
  int sh = max(0, 32 - __builtin_clz(f.lim | 1u) - 6);
  if (((f.lim + (1u << sh) - 1u) >> sh) > uint32_t(kStRefineBins)) ++sh;
  f.sh = sh;
  f.pad = (0u - f.lim) & ((1u << sh) - 1u);
  return f;
}

// f(u) for the lane's n column values (raw float bits) in row order.
// U loads in flight per lane (the kernel's LDS caps it at 2 waves
// per SIMD, so the bytes in flight per CU come from this depth); the last
// partial batch re-reads row n - 1 in its unused slots and skips them.
typedef __attribute__((address_space(1))) const uint32_t gu32;
__device__ __forceinline__ uint32_t col_at(const float *const *rows, int j,
                                           uint32_t off) {
  return *(gu32 *)((gchar *)row_at(rows, j) + off * 4u);
}

template <int U, typename F>
__device__ __forceinline__ void stream_column(const float *const *rows, int n,
                                              uint32_t off, F &&f) {
  int j = 0;
#pragma unroll 1
  for (; j + U <= n; j += U) {
    uint32_t u[U];
#pragma unroll
    for (int i = 0; i < U; ++i) u[i] = col_at(rows, j + i, off);
#pragma unroll
    for (int i = 0; i < U; ++i) f(u[i]);
  }
  if (j < n) {
    uint32_t u[U];
#pragma unroll
    for (int i = 0; i < U; ++i) u[i] = col_at(rows, min(j + i, n - 1), off);
#pragma unroll
    for (int i = 0; i < U; ++i)
      if (j + i < n) f(u[i]);
  }
}

// stream_column from the last row down: the pass after a forward pass
// starts on the rows that pass read last, which the XCD's L2 may still hold
template <int U, typename F>
__device__ __forceinline__ void stream_column_rev(const float *const *rows,
                                                  int n, uint32_t off,
                                                  F &&f) {
  int j = n;
#pragma unroll 1
  for (; j - U >= 0; j -= U) {
    uint32_t u[U];
#pragma unroll
    for (int i = 0; i < U; ++i) u[i] = col_at(rows, j - 1 - i, off);
#pragma unroll
    for (int i = 0; i < U; ++i) f(u[i]);
  }
  if (j > 0) {
    uint32_t u[U];
#pragma unroll
    for (int i = 0; i < U; ++i) u[i] = col_at(rows, max(j - 1 - i, 0), off);
#pragma unroll
    for (int i = 0; i < U; ++i)
      if (j - 1 - i >= 0) f(u[i]);
  }
}

template <int MODE, int U>
__global__ __launch_bounds__(kBlock) void orderstat_stream_kernel(
    RowSrc rs, int n, int kk, float divisor, float *__restrict__ out) {
  __shared__ __attribute__((aligned(16384))) uint32_t lds[kSelLds];
  uint32_t *H = lds + (threadIdx.x / kWave) * kSelWords * kWave +
                (threadIdx.x & (kWave - 1));
  const uint32_t hb = uint32_t(uintptr_t((lds_u32 *)H));
  const BlockRows br = block_rows(rs, blockIdx.x);
  const float *const *__restrict__ rows = br.rows;
  const int64_t p = br.lo + threadIdx.x;
  const bool live = int(threadIdx.x) < br.len;
  // coordinates < 2^30 (launch); dead lanes re-read the chunk's first
  const uint32_t off = uint32_t(live ? p : br.lo);

  // 1. the digit's reference magnitude: the largest finite |x| of the
  // first kStSample rows.  Any base gives exact bins (the top digit runs
  // up to +-inf, the bottom one down to 0), the sample only sets how finely
  // the bulk is split; values above it land in the top bins.
  uint32_t smax = 0u;
  const float bval = br.base ? ld_nt(br.base, off) : 0.0f;
  stream_column<U>(rows, min(n, kStSample), off, [&](uint32_t u) {
    const uint32_t a = u & 0x7FFFFFFFu;
    smax = a < 0x7F800000u ? max(smax, a) : smax;
  });
  const int obase = int(smax >> kStMagShift) - (kStCodes - 1);
  const int r1 = MODE == kMedian ? (n - 1) / 2 : kk;
  const int r2 = MODE == kMedian ? n / 2 : n - kk - 1;

  // 2. octave-digit histogram: both ranks' bins (and NaN/inf over all rows)
  RankSel s1, s2;
  uint32_t amax = 0u;
  {
    hist_clear(H, 64);
    stream_column<U>(rows, n, off, [&](uint32_t u) {
      amax = max(amax, u & 0x7FFFFFFFu);
      hist16_inc(hb, st_digit(u, obase));
    });
    uint32_t d1, d2;
    int b1, c1, b2, c2;
    hist16_find2(H, r1, r2, d1, b1, c1, d2, b2, c2);
    st_bin(d1, obase, s1.lo, s1.hi);
    st_bin(d2, obase, s2.lo, s2.hi);
    s1.below = b1;
    s1.cnt = c1;
    s2.below = b2;
    s2.cnt = c2;
  }
  const bool nan = amax > 0x7F800000u;
  const bool nonfinite = amax >= 0x7F800000u;

  // 3. refine while the two bins would overflow the list
  bool shared = same_bin(s1, s2);
#pragma unroll 1
  for (int round = 0; round < 12; ++round) {
    const bool list1 = !resolved(s1), list2 = !shared && !resolved(s2);
    const int stored = (list1 ? s1.cnt : 0) + (list2 ? s2.cnt : 0);
    const bool need = stored > kList;
    if (!__any(need)) break;
    const bool pick2 = list2 && (!list1 || s2.cnt > s1.cnt);
    const Refine f = st_refine_plan(pick2 ? s2 : s1);
    hist_clear(H, 33);
    stream_column<U>(rows, n, off, [&](uint32_t u) {
      const uint32_t rel = min(ukey(u) - f.lo, f.lim);
      hist16_inc(hb, (rel + f.pad) >> f.sh);
    });
    uint32_t da, db;
    int ba, ca, bb, cb;
    const int ra = pick2 ? r2 - s2.below : r1 - s1.below;
    hist16_find2(H, ra, r2 - s2.below, da, ba, ca, db, bb, cb);
    refine_apply(s2, f, need && shared, db, bb, cb);
    refine_apply(s2, f, need && pick2, da, ba, ca);
    refine_apply(s1, f, need && !pick2, da, ba, ca);
    shared = same_bin(s1, s2);
  }

  // 4. compaction: the listed bins' values (at most kList), the rows read
  // last first (stream_column_rev; the list is sorted afterwards)
  const bool list1 = !resolved(s1);
  const bool list2 = !shared && !resolved(s2);
  double mid = 0.0;
  if (__any(list1 || list2) || MODE == kTrimmed) {
    int c = 0;
    if constexpr (MODE == kMedian) {
      // ranks r1, r1 + 1 are adjacent: one key range [lo, lo + w) covers
      // both lists
      const uint32_t lo = list1 ? s1.lo : s2.lo;
      const uint32_t w =
          (list1 || list2) ? (list2 ? s2.hi : s1.hi) - lo + 1u : 0u;
      stream_column_rev<U>(rows, n, off, [&](uint32_t u) {
        *lds_at(hb | (uint32_t(c) << 8)) = u;  // a miss: overwritten
        c = add_below(c, ukey(u) - lo, w);
      });
    } else {
      const uint32_t A = list1 ? s1.lo : s1.hi + 1u;
      const uint32_t w1 = list1 ? s1.hi - s1.lo + 1u : 0u;
      const uint32_t wm = shared ? 0u : s2.lo - (s1.hi + 1u);
      const uint32_t wb = w1 + wm + (list2 ? s2.hi - s2.lo + 1u : 0u);
      stream_column_rev<U>(rows, n, off, [&](uint32_t u) {
        const uint32_t rel = ukey(u) - A;
        const bool inm = rel - w1 < wm;
        float x = inm ? __uint_as_float(u) : 0.0f;
        asm("" : "+v"(x));
        mid += double(x);
        *lds_at(hb | (uint32_t(c) << 8)) = u;  // a miss: overwritten
        c += (rel < wb) && !inm;
      });
    }
  }

  // 5. the ranks (and the kept sum) off the sorted list
  constexpr bool SUM = MODE == kTrimmed;
  const int rr1 = r1 - s1.below, rr2 = r2 - s2.below;
  const int c1off = list1 ? s1.cnt : 0;
  const int stored = c1off + (list2 ? s2.cnt : 0);
  const int pb = shared ? rr2 : c1off + rr2;
  int lo, hi;
  double fixed = 0.0;
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
    r = __fdiv_rn(key2f(v1) - (-key2f(v2)), 2.0f);
    if (nan) r = __builtin_nanf("");
  } else {
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
  if (br.base) r = add_rn(bval, r);
  out[p] = r;
}

}  // namespace

// rows in flight per lane: 32 (16: 5-10 % slower on the trimmed mean; 64:
// no gain)
constexpr int kStreamUnroll = 32;

template <int MODE>
void launch_stream(const RowSrc &rs, unsigned grid, int n, int kk,
                   float divisor, float *out, hipStream_t s) {
  hipLaunchKernelGGL((orderstat_stream_kernel<MODE, kStreamUnroll>),
                     dim3(grid), dim3(kBlock), 0, s, rs, n, kk, divisor, out);
}

template void launch_stream<kMedian>(const RowSrc &, unsigned, int, int,
                                     float, float *, hipStream_t);
template void launch_stream<kTrimmed>(const RowSrc &, unsigned, int, int,
                                      float, float *, hipStream_t);

}  // namespace os
}  // namespace fsagg
