// Internal to libfsagg: device helpers shared by the order-statistics
// translation units (orderstat.hip and the per-N orderstat_select.hip
// instantiations).  Not part of the public ABI.
#pragma once

#include <atomic>
#include <utility>

#include "common.h"

namespace fsagg {
namespace os {

// Non-temporal global load at a 32-bit element offset from a row base (each
// column value is read once).
// The byte offset is formed in 32 bits and zero-extended, so the load takes
// the SGPR-base + 32-bit VGPR-offset form (global_load_dword v, v_off, s[b])
// with no per-row 64-bit address add.  Callers keep off < 2^30.
typedef __attribute__((address_space(1))) const float gfloat;
typedef __attribute__((address_space(1))) const char gchar;
__device__ __forceinline__ float ld_nt(const float *row, uint32_t off) {
  const uint32_t boff = off * 4u;
  return __builtin_nontemporal_load(
      (gfloat *)((gchar *)(row) + boff));
}

// Row pointer j of a device row table, read through the constant address
// space: the table is never written while a kernel runs, so the load stays a
// scalar s_load even in a loop that also stores to global memory (a plain
// load there becomes a vector load + v_readfirstlane per row).
typedef const float *const __attribute__((address_space(4))) const_row_t;
__device__ __forceinline__ const float *row_at(const float *const *tab,
                                               int j) {
  return ((const_row_t *)(tab))[j];
}

constexpr int kBlock = 256;
constexpr uint32_t kPad = 0xFFFFFFFFu;

// ---- compile-time sorting network (Batcher's odd-even merge sort) -------
// Ascending; N a power of two.  191 compare-exchanges at N = 32 and 543 at
// N = 64, against 240 / 672 for the bitonic network (each one v_min_u32 +
// v_max_u32).  Stage (P, Q) compares i + j with i + j + Q inside the same
// 2P-block; P and Q are template constants, so every loop below unrolls to
// constant register indices.
template <int N, int P, int Q>
__device__ __forceinline__ void oem_stage(uint32_t (&k)[N]) {
#pragma unroll
  for (int j = Q % P; j + Q < N; j += 2 * Q) {
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      if (i + j + Q < N && (i + j) / (2 * P) == (i + j + Q) / (2 * P)) {
        const uint32_t a = k[i + j], b = k[i + j + Q];
        k[i + j] = a < b ? a : b;
        k[i + j + Q] = a < b ? b : a;
      }
    }
  }
  if constexpr (Q > 1) oem_stage<N, P, Q / 2>(k);
}

template <int N, int P>
__device__ __forceinline__ void oem_from(uint32_t (&k)[N]) {
  oem_stage<N, P, P>(k);
  if constexpr (2 * P < N) oem_from<N, 2 * P>(k);
}

template <int N>
__device__ __forceinline__ void sort_network(uint32_t (&k)[N]) {
  static_assert(N >= 2 && (N & (N - 1)) == 0, "N: a power of two");
  oem_from<N, 1>(k);
}

// The same network as a comparator list, pruned to the comparators that can
// reach output positions [LO, HI] (backward liveness: a comparator is kept
// when either of its outputs is live, and then both its inputs are).  The
// values at [LO, HI] are exactly the sorted ones; the rest are not sorted.
// The median reads two positions: at N = 32 this keeps 169 of 191
// comparators, at N = 64 (positions 16..32) 477 of 543.
template <int N>
constexpr int oem_count() {
  int c = 0;
  for (int p = 1; p < N; p <<= 1)
    for (int q = p; q >= 1; q >>= 1)
      for (int j = q % p; j + q < N; j += 2 * q)
        for (int i = 0; i < q; ++i)
          if (i + j + q < N && (i + j) / (2 * p) == (i + j + q) / (2 * p)) ++c;
  return c;
}

template <int N>
struct OemNet {
  static constexpr int C = oem_count<N>();
  int a[C], b[C];
  bool keep[C];
  constexpr OemNet(int lo, int hi) : a{}, b{}, keep{} {
    int c = 0;
    for (int p = 1; p < N; p <<= 1)
      for (int q = p; q >= 1; q >>= 1)
        for (int j = q % p; j + q < N; j += 2 * q)
          for (int i = 0; i < q; ++i)
            if (i + j + q < N && (i + j) / (2 * p) == (i + j + q) / (2 * p)) {
              a[c] = i + j;
              b[c] = i + j + q;
              ++c;
            }
    bool live[N] = {};
    for (int x = lo; x <= hi; ++x) live[x] = true;
    for (int t = C - 1; t >= 0; --t) {
      keep[t] = live[a[t]] || live[b[t]];
      if (keep[t]) live[a[t]] = live[b[t]] = true;
    }
  }
};

__device__ __forceinline__ void cas_up(uint32_t &x, uint32_t &y) {
  const uint32_t a = x, b = y;
  x = a < b ? a : b;
  y = a < b ? b : a;
}

template <int N, int LO, int HI, int... T>
__device__ __forceinline__ void oem_pruned(uint32_t (&k)[N],
                                           std::integer_sequence<int, T...>) {
  constexpr OemNet<N> net(LO, HI);
  ((net.keep[T] ? cas_up(k[net.a[T]], k[net.b[T]]) : void()), ...);
}

// positions [LO, HI] of the sorted keys, the rest unordered
template <int N, int LO, int HI>
__device__ __forceinline__ void select_network(uint32_t (&k)[N]) {
  static_assert(0 <= LO && LO <= HI && HI < N, "positions");
  oem_pruned<N, LO, HI>(k, std::make_integer_sequence<int, OemNet<N>::C>{});
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
  // select in fp32, then widen: one v_cndmask, not a 64-bit pair (the empty
  // asm keeps the compiler from sinking the select past the cvt)
  auto term = [&](int i) {
    float x = (i >= lo && i < hi) ? key2f(k[i]) : 0.0f;
    asm("" : "+v"(x));
    return double(x);
  };
  ((s += term(I)), ...);
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

// Where a block's coordinates and clients live.  Flat form (chunks ==
// nullptr): block b covers [b·kBlock, …) of [0, numel) and client j's row
// is tab[j]; row-set form (include/fsagg.h fsagg_rows): block b is chunk b
// (one key segment, <= kBlock coordinates) and client j's row of segment
// seg is tab[seg·ss + j] (a virtual base: coordinate p is row[p]).
struct RowSrc {
  const float *const *tab;
  int64_t ss;
  const fsagg_chunk *chunks;
  int64_t numel;
  const float *base;          // flat base (tab form), or
  const float *const *btab;   // per-segment virtual bases, stride bss
  int64_t bss;
};

struct BlockRows {
  const float *const *rows;  // client j: rows[j]
  int64_t lo;                // first coordinate
  int len;                   // live lanes
  const float *base;
};

__device__ __forceinline__ BlockRows block_rows(const RowSrc &rs, int b) {
  BlockRows br;
  int seg = 0;
  if (rs.chunks) {
    br.lo = rs.chunks[b].lo;
    br.len = rs.chunks[b].len;
    seg = rs.chunks[b].seg;
  } else {
    br.lo = int64_t(b) * kBlock;
    const int64_t r = rs.numel - br.lo;
    br.len = r < kBlock ? int(r) : kBlock;
  }
  br.rows = rs.tab + int64_t(seg) * rs.ss;
  br.base = rs.btab ? rs.btab[int64_t(seg) * rs.bss] : rs.base;
  return br;
}

inline unsigned rows_grid(const RowSrc &rs, int nchunk) {
  return rs.chunks ? unsigned(nchunk)
                   : unsigned((rs.numel + kBlock - 1) / kBlock);
}


// The select kernel for register-array size N serves N - kSelStep < n <= N.
constexpr int kSelStep = 8;

// Launch the range-adaptive select kernel for 64 < n <= N (orderstat_select.hip,
// one translation unit per N).
template <int N, int MODE>
void launch_select(const RowSrc &rs, unsigned grid, int n, int kk,
                   float divisor, float *out, hipStream_t s);

// Default client count from which 64 < n <= 255 runs the two-wave kernel.
constexpr int kPairMinDefault = 129;

// Launch the two-wave select kernel for 2H - 8 < n <= 2H (orderstat_pair.h,
// built in orderstat_select.hip's translation unit for SEL_N = 2H); its grid
// is one 128-thread block per 64 coordinates.
template <int H, int MODE>
void launch_pair(const RowSrc &rs, unsigned grid, int n, int kk, float divisor,
                 float *out, hipStream_t s);

// Launch the K-wave select kernel (orderstat_group.h) for 255 < n <= 512;
// false when n is outside its range (the caller streams instead).  Its grid
// is one block of K·64 threads per 64 coordinates, as launch_pair's.
template <int MODE>
bool launch_group(const RowSrc &rs, unsigned grid, int n, int kk,
                  float divisor, float *out, hipStream_t s);
// its waves per block (fsagg_orderstat_set_group_waves)
extern std::atomic<int> g_group_waves;

// Launch the streaming select kernel for 255 < n <= 65535
// (orderstat_stream.hip).
template <int MODE>
void launch_stream(const RowSrc &rs, unsigned grid, int n, int kk,
                   float divisor, float *out, hipStream_t s);

}  // namespace os
}  // namespace fsagg
