// FedAvg-family weighted sum over client buckets (gfx950).
//
// Semantics: ClientsAvgAggregator._para_weighted_avg
// (federatedscope/core/aggregators/clients_avg_aggregator.py:60-100): per
// element, acc = x0*w0, then acc = acc + xi*wi in client-list order, every
// multiply and add rounded to fp32 separately (ATen CPU semantics; no FMA).
//
// HBM layout: each client's update is one flat fp32 bucket (a row); the
// kernel reads a row table so stacked slabs, per-client tensors and Krum's
// selected subsets all stream without a gather copy.  Bytes per element:
// 4·n read + 4 written (+4 read for the fused `base` add) — the whole kernel
// is HBM-bound (0.5 FLOP/B), so the design goal is pure streaming:
//   * each thread owns V float4 columns of the bucket (16 B/lane, 1 KiB per
//     wave-instruction per row, fully coalesced), V up to 24: 384 B of one
//     client row in flight per lane before any of it is consumed;
//   * the adds happen strictly in client order, which keeps the result
//     bit-identical to the reference;
//   * row pointers and weights are wave-uniform → scalar (SGPR) loads.
#include <atomic>
#include <hip/hip_fp16.h>

#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;

// clang ext-vector (the nontemporal builtin needs a native vector type)
typedef float f4 __attribute__((ext_vector_type(4)));

// Row pointers arrive through a table, so the compiler cannot prove they are
// global memory and would emit flat loads; cast to the global address space
// (addrspace 1) so the streaming loads are global_load_dwordx4 (nt).
typedef __attribute__((address_space(1))) const f4 gf4;

template <bool NT>
__device__ __forceinline__ f4 ld4(const f4 *p) {
  gf4 *g = (gf4 *)(p);
  if constexpr (NT) {
    return __builtin_nontemporal_load(g);
  } else {
    return *g;
  }
}

// One client's chunk row as a raw buffer (wave-uniform base and byte count):
// each 16-B load is buffer_load_dwordx4 v_off, s[rsrc], s_off nt — the lane
// offset in one VGPR and the per-v displacement on the scalar side, where
// global loads of a table-held row pointer need a 64-bit VALU add (and its
// VCC carry) per load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const float *p,
                                                           int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), short(0),
                                           bytes, 0x00020000);
}
__device__ __forceinline__ f4 ld4_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                      uint32_t soff) {
  // aux 2: non-temporal (streamed once)
  return __builtin_bit_cast(
      f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 2));
}
// f4 column v of a chunk row: a whole chunk puts the displacement in the
// scalar offset; a partial chunk (GUARD) keeps it in the vector offset, the
// part of the address the range check covers, so columns past the chunk
// read 0 instead of whatever follows it
template <bool GUARD>
__device__ __forceinline__ f4 ld4_rowv(__amdgpu_buffer_rsrc_t r,
                                       uint32_t loff, int v) {
  const uint32_t d = uint32_t(v) * uint32_t(kBlock) * 16u;
  return GUARD ? ld4_buf(r, loff + d, 0u) : ld4_buf(r, loff, d);
}

__device__ __forceinline__ f4 mul4(f4 a, float s) {
  return f4{mul_rn(a.x, s), mul_rn(a.y, s), mul_rn(a.z, s), mul_rn(a.w, s)};
}
__device__ __forceinline__ f4 add4(f4 a, f4 b) {
  return f4{add_rn(a.x, b.x), add_rn(a.y, b.y), add_rn(a.z, b.z),
            add_rn(a.w, b.w)};
}

// One tile of V f4 columns per thread.  GUARD handles the ragged last
// tile; all other tiles run unguarded.
// Output of a tile: one bucket (float *), or the same coordinates of up to
// kMaxPeers buckets — every GPU's copy of the assembled result, peers' over
// xGMI (fsagg_weighted_sum_bcast_f32).
struct Bcast {
  float *p[FSAGG_MAX_PEERS];
  int n;
};
__device__ __forceinline__ void put4(float *out, int64_t i, f4 a) {
  reinterpret_cast<f4 *>(out)[i] = a;
}
__device__ __forceinline__ void put4(const Bcast &o, int64_t i, f4 a) {
#pragma unroll
  for (int k = 0; k < FSAGG_MAX_PEERS; ++k)
    if (k < o.n) reinterpret_cast<f4 *>(o.p[k])[i] = a;
}

template <int U, int V, bool PRE, bool BASE, bool NT, bool GUARD, class O>
__device__ __forceinline__ void wsum_tile(const float *const *__restrict__ rows,
                                          const float *__restrict__ w,
                                          const float *__restrict__ pre, int n,
                                          int64_t nvec, int64_t t0,
                                          const float *__restrict__ base,
                                          const O &out) {
  int64_t idx[V];
  bool ok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    idx[v] = t0 + v * kBlock + threadIdx.x;
    ok[v] = !GUARD || idx[v] < nvec;
  }
  f4 acc[V];
  // client 0 initialises the accumulator (the reference's i == 0 branch)
  {
    const f4 *r = reinterpret_cast<const f4 *>(rows[0]);
    const float w0 = w[0];
    const float s0 = PRE ? pre[0] : 1.0f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      f4 x = ok[v] ? ld4<NT>(r + idx[v]) : f4{0.0f, 0.0f, 0.0f, 0.0f};
      if (PRE) x = mul4(x, s0);
      acc[v] = mul4(x, w0);
    }
  }
  int i = 1;
  for (; i + U <= n; i += U) {
    f4 x[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f4 *r = reinterpret_cast<const f4 *>(rows[i + u]);
#pragma unroll
      for (int v = 0; v < V; ++v)
        x[u][v] = ok[v] ? ld4<NT>(r + idx[v]) : f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float wu = w[i + u];
      const float su = PRE ? pre[i + u] : 1.0f;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        f4 t = x[u][v];
        if (PRE) t = mul4(t, su);
        acc[v] = add4(acc[v], mul4(t, wu));
      }
    }
  }
  for (; i < n; ++i) {
    const f4 *r = reinterpret_cast<const f4 *>(rows[i]);
    const float wi = w[i];
    const float si = PRE ? pre[i] : 1.0f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      f4 t = ok[v] ? ld4<NT>(r + idx[v]) : f4{0.0f, 0.0f, 0.0f, 0.0f};
      if (PRE) t = mul4(t, si);
      acc[v] = add4(acc[v], mul4(t, wi));
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (!ok[v]) continue;
    f4 a = acc[v];
    if (BASE) a = add4(reinterpret_cast<const f4 *>(base)[idx[v]], a);
    put4(out, idx[v], a);
  }
}

template <int U, int V, bool PRE, bool BASE, bool NT, class O = float *>
__global__ __launch_bounds__(kBlock) void wsum_f32_vec_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w,
    const float *__restrict__ pre, int n, int64_t nvec,
    const float *__restrict__ base, O out) {
  constexpr int64_t tile = int64_t(kBlock) * V;
  const int64_t full = nvec / tile * tile;
  for (int64_t t0 = int64_t(blockIdx.x) * tile; t0 < nvec;
       t0 += int64_t(gridDim.x) * tile) {
    if (t0 < full)
      wsum_tile<U, V, PRE, BASE, NT, false>(rows, w, pre, n, nvec, t0, base,
                                            out);
    else
      wsum_tile<U, V, PRE, BASE, NT, true>(rows, w, pre, n, nvec, t0, base,
                                           out);
  }
}

// Block-contiguous partition: block b streams float4 columns
// [b·chunk, (b+1)·chunk) in tiles of kBlock·V.  With grid = (resident blocks
// per CU) × 256 every CU gets the same byte count, so no CU idles through a
// tail wave while the others finish (the tile-granular grid-stride form
// leaves up to one tile-round of imbalance).
template <int U, int V, bool PRE, bool BASE, bool NT>
__global__ __launch_bounds__(kBlock) void wsum_f32_part_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w,
    const float *__restrict__ pre, int n, int64_t nvec, int64_t chunk,
    const float *__restrict__ base, float *__restrict__ out) {
  constexpr int64_t tile = int64_t(kBlock) * V;
  const int64_t lo = int64_t(blockIdx.x) * chunk;
  const int64_t hi = lo + chunk < nvec ? lo + chunk : nvec;
  for (int64_t t0 = lo; t0 < hi; t0 += tile) {
    if (t0 + tile <= hi)
      wsum_tile<U, V, PRE, BASE, NT, false>(rows, w, pre, n, hi, t0, base,
                                            out);
    else
      wsum_tile<U, V, PRE, BASE, NT, true>(rows, w, pre, n, hi, t0, base,
                                           out);
  }
}

// Scalar tail: elements [start, numel) (fewer than 4), one thread each.
__device__ __forceinline__ void put1(float *out, int64_t p, float a) {
  out[p] = a;
}
__device__ __forceinline__ void put1(const Bcast &o, int64_t p, float a) {
  for (int k = 0; k < o.n; ++k) o.p[k][p] = a;
}
// The < 4 elements past the last float4 column.  One block: the n client
// values of each tail element are loaded 256 clients at a time by all the
// threads together (one memory latency per 256 clients, where a single
// thread walking the clients waited out n dependent loads: 45 us at n =
// 100), then thread e adds them up for element e in client order from LDS.
constexpr int kTailBlock = 256;
template <class O = float *>
__global__ __launch_bounds__(kTailBlock) void wsum_f32_tail_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w,
    const float *__restrict__ pre, int n, int64_t start, int64_t numel,
    const float *__restrict__ base, O out) {
  __shared__ float xs[3][kTailBlock];
  const int m = int(numel - start);  // 1..3
  const int e = threadIdx.x;
  float acc = 0.0f;
  for (int c0 = 0; c0 < n; c0 += kTailBlock) {
    const int c = c0 + threadIdx.x;
    if (c < n) {
      const float *r = rows[c];
      const float s = pre ? pre[c] : 1.0f;
      for (int k = 0; k < m; ++k) {
        float x = gld(r + start + k);
        if (pre) x = mul_rn(x, s);
        xs[k][threadIdx.x] = x;
      }
    }
    __syncthreads();
    if (e < m) {
      const int cn = n - c0 < kTailBlock ? n - c0 : kTailBlock;
      for (int j = 0; j < cn; ++j) {
        const float t = mul_rn(xs[e][j], w[c0 + j]);
        acc = c0 + j == 0 ? t : add_rn(acc, t);
      }
    }
    __syncthreads();
  }
  if (e < m) {
    const int64_t p = start + e;
    if (base) acc = add_rn(base[p], acc);
    put1(out, p, acc);
  }
}

// Launch shape of the streaming kernel, from interleaved timing on MI355X
// (tools/tune_wsum.py; profiles/r01_tune_wsum_box*.txt).  One client row in
// flight (U = 1) and V float4 columns per lane; V is the largest that still
// gives >= ~1000 one-tile workgroups (≈ 2 rounds of the 2 × 256 resident
// workgroups at the ~200 VGPRs V = 24 needs).  At 100 × 25M that is V = 24,
// 1018 workgroups: 1.43–1.45 ms = 6.95–7.08 TB/s on two boxes, above the
// chip's plain nt read stream (6.5–6.7 TB/s); V = 20 (1221 workgroups,
// a ragged third round) loses 25 %.
constexpr int kU = 1;

template <bool PRE, bool BASE, int V, class O>
void launch_wsum_v(const float *const *rows, const float *w, const float *pre,
                   int n, int64_t nvec, const float *base, O out,
                   hipStream_t s) {
  const int64_t tiles = (nvec + int64_t(kBlock) * V - 1) / (int64_t(kBlock) * V);
  const unsigned grid = stream_grid(tiles, 1, 256 * 16);
  hipLaunchKernelGGL((wsum_f32_vec_kernel<kU, V, PRE, BASE, true, O>),
                     dim3(grid), dim3(kBlock), 0, s, rows, w, pre, n, nvec,
                     base, out);
}

// V of the row-set kernel's chunks (wsum_rows_kernel) for nvec float4
// columns of n clients: the largest V that leaves >= min_tiles one-tile
// workgroups.  1000 (two rounds of the 2 × 256 resident workgroups) below
// 150 clients; with n >= 150 a tile runs long enough that ~400 workgroups
// keep HBM busy and the wider V wins: 200 × 6.6M, V = 16 (403 tiles)
// 0.79 ms against V = 4 (1612) 0.83 ms and V = 24 (269) 1.06 ms
// (profiles/r02_tune_wsum_200x6p6M.txt).
inline int wsum_width_rows(int64_t nvec, int n) {
  const int64_t min_tiles = n >= 150 ? 400 : 1000;
  auto tiles = [&](int v) { return (nvec + 256 * v - 1) / (256 * v); };
  for (int v : {24, 16, 8, 4})
    if (tiles(v) >= min_tiles) return v;
  return 1;
}

// V of the flat streaming kernels (wsum_f32_vec_kernel, the host-table
// kernel).  Fitted to an interleaved sweep of V = 1/4/8/12/16/24 over
// 1.69M–50M coordinates at n = 30/50/100/200 (tools/tune_wsum.py,
// profiles/r06/tune_wsum_sizes_*.txt; 256-B aligned rows).  V = 24 (244
// VGPRs, two workgroups per CU: 512 resident) wins whenever its last round
// of workgroups is at least half full — r = tiles/512 >= 0.9 with
// frac(r) >= 0.5 (12M: 0.680 against 0.733 ms for V = 16; 23.5M: 1.357
// against 1.442; 25M; 32M; 50M) — and loses up to 20 % when that round is
// mostly empty (15M, r = 1.19: 1.141 against 0.950; 28M, r = 2.22: 1.866
// against 1.746).  Otherwise V = 16 (164 VGPRs, three per CU) from 400
// tiles up or while its tiles fit one per CU from 160 (3M: 0.170 ms against
// 0.193 for V = 1; at 305 tiles, 5M, the CUs holding two take twice as
// long: 0.366 against 0.317 for V = 4); then V = 4 from 1000 tiles, V = 8
// from 200 (1.69M: 0.097 against 0.103 for V = 1), else V = 1.  The choice
// never changes a result bit: each element sums its clients in order.
inline int wsum_width(int64_t nvec, int n) {
  (void)n;
  auto tiles = [&](int v) { return (nvec + 256 * v - 1) / (256 * v); };
  const double r = double(tiles(24)) / 512.0;
  if (r >= 0.9 && r - double(int64_t(r)) >= 0.5) return 24;
  const int64_t t16 = tiles(16);
  if (t16 >= 400 || (t16 >= 160 && t16 <= 256)) return 16;
  if (tiles(4) >= 1000) return 4;
  if (tiles(8) >= 200) return 8;
  return 1;
}

template <bool PRE, bool BASE, class O>
void launch_wsum(const float *const *rows, const float *w, const float *pre,
                 int n, int64_t nvec, const float *base, O out,
                 hipStream_t s) {
  switch (wsum_width(nvec, n)) {
    case 24: launch_wsum_v<PRE, BASE, 24>(rows, w, pre, n, nvec, base, out, s); break;
    case 16: launch_wsum_v<PRE, BASE, 16>(rows, w, pre, n, nvec, base, out, s); break;
    case 8: launch_wsum_v<PRE, BASE, 8>(rows, w, pre, n, nvec, base, out, s); break;
    case 4: launch_wsum_v<PRE, BASE, 4>(rows, w, pre, n, nvec, base, out, s); break;
    default: launch_wsum_v<PRE, BASE, 1>(rows, w, pre, n, nvec, base, out, s);
  }
}

template <class O>
void launch_wsum_any(const float *const *rows, const float *weights,
                     const float *prescale, int n, int64_t numel,
                     const float *base, O out, hipStream_t s) {
  const int64_t nvec = numel / 4;
  if (nvec > 0) {
    if (prescale) {
      if (base) launch_wsum<true, true>(rows, weights, prescale, n, nvec, base, out, s);
      else launch_wsum<true, false>(rows, weights, prescale, n, nvec, base, out, s);
    } else {
      if (base) launch_wsum<false, true>(rows, weights, prescale, n, nvec, base, out, s);
      else launch_wsum<false, false>(rows, weights, prescale, n, nvec, base, out, s);
    }
  }
  if (numel > nvec * 4) {
    hipLaunchKernelGGL((wsum_f32_tail_kernel<O>), dim3(1), dim3(kTailBlock),
                       0, s, rows, weights, prescale, n, nvec * 4, numel, base,
                       out);
  }
}

// ---------------------------------------------------------------------------
// Host tables in the kernel arguments (fsagg_weighted_sum_hosttab_f32): up
// to FSAGG_HOSTTAB_MAX_CLIENTS row pointers, weights and prescales travel in
// the launch's kernel-argument block (2 KiB), which the kernels read with
// scalar loads exactly as they read a device table — no upload, no copy on
// any stream before the launch.  The aggregate() path for a flat or uniform
// row set of fresh uploads (new tensors every round) spends most of its
// host time on those small uploads otherwise.
// ---------------------------------------------------------------------------
static_assert(FSAGG_HOSTTAB_MAX_CLIENTS <= 256,
              "the host-table tail kernel loads one client per thread");
struct ArgTab {
  const float *rows[FSAGG_HOSTTAB_MAX_CLIENTS];
  float w[FSAGG_HOSTTAB_MAX_CLIENTS];
  float pre[FSAGG_HOSTTAB_MAX_CLIENTS];
};

template <int U, int V, bool PRE, bool BASE, bool NT, class O>
__global__ __launch_bounds__(kBlock) void wsum_f32_arg_kernel(
    const ArgTab tab, int n, int64_t nvec, const float *__restrict__ base,
    O out) {
  constexpr int64_t tile = int64_t(kBlock) * V;
  const int64_t full = nvec / tile * tile;
  for (int64_t t0 = int64_t(blockIdx.x) * tile; t0 < nvec;
       t0 += int64_t(gridDim.x) * tile) {
    if (t0 < full)
      wsum_tile<U, V, PRE, BASE, NT, false>(tab.rows, tab.w, tab.pre, n, nvec,
                                            t0, base, out);
    else
      wsum_tile<U, V, PRE, BASE, NT, true>(tab.rows, tab.w, tab.pre, n, nvec,
                                           t0, base, out);
  }
}

template <class O>
__global__ __launch_bounds__(kTailBlock) void wsum_f32_arg_tail_kernel(
    const ArgTab tab, int pre_on, int n, int64_t start, int64_t numel,
    const float *__restrict__ base, O out) {
  // n <= FSAGG_HOSTTAB_MAX_CLIENTS < kTailBlock: thread c loads client c's
  // (<= 3) tail values into LDS — one memory latency for all clients (a
  // thread walking the clients waited out their loads one by one: 46 us at
  // n = 100, profiles/r06/layout_b_trace) — then thread e sums element e in
  // client order
  __shared__ float xs[3][kTailBlock];
  const int m = int(numel - start);  // 1..3
  const int c = threadIdx.x;
  if (c < n) {
    const float *r = tab.rows[c];
    const float sc = pre_on ? tab.pre[c] : 1.0f;
    for (int k = 0; k < m; ++k) {
      float x = gld(r + start + k);
      if (pre_on) x = mul_rn(x, sc);
      xs[k][c] = x;
    }
  }
  __syncthreads();
  const int e = threadIdx.x;
  if (e >= m) return;
  float acc = 0.0f;
  for (int j = 0; j < n; ++j) {
    const float t = mul_rn(xs[e][j], tab.w[j]);
    acc = j == 0 ? t : add_rn(acc, t);
  }
  if (base) acc = add_rn(base[start + e], acc);
  put1(out, start + e, acc);
}

template <bool PRE, bool BASE, int V, class O>
void launch_wsum_arg_v(const ArgTab &tab, int n, int64_t nvec,
                       const float *base, O out, hipStream_t s) {
  const int64_t tiles = (nvec + int64_t(kBlock) * V - 1) / (int64_t(kBlock) * V);
  const unsigned grid = stream_grid(tiles, 1, 256 * 16);
  hipLaunchKernelGGL((wsum_f32_arg_kernel<kU, V, PRE, BASE, true, O>),
                     dim3(grid), dim3(kBlock), 0, s, tab, n, nvec, base, out);
}

template <bool PRE, bool BASE, class O>
void launch_wsum_arg(const ArgTab &tab, int n, int64_t nvec,
                     const float *base, O out, hipStream_t s) {
  switch (wsum_width(nvec, n)) {
    case 24: launch_wsum_arg_v<PRE, BASE, 24>(tab, n, nvec, base, out, s); break;
    case 16: launch_wsum_arg_v<PRE, BASE, 16>(tab, n, nvec, base, out, s); break;
    case 8: launch_wsum_arg_v<PRE, BASE, 8>(tab, n, nvec, base, out, s); break;
    case 4: launch_wsum_arg_v<PRE, BASE, 4>(tab, n, nvec, base, out, s); break;
    default: launch_wsum_arg_v<PRE, BASE, 1>(tab, n, nvec, base, out, s);
  }
}

template <class O>
void launch_wsum_arg_any(const ArgTab &tab, bool pre, int n, int64_t numel,
                         const float *base, O out, hipStream_t s) {
  const int64_t nvec = numel / 4;
  if (nvec > 0) {
    if (pre) {
      if (base) launch_wsum_arg<true, true>(tab, n, nvec, base, out, s);
      else launch_wsum_arg<true, false>(tab, n, nvec, base, out, s);
    } else {
      if (base) launch_wsum_arg<false, true>(tab, n, nvec, base, out, s);
      else launch_wsum_arg<false, false>(tab, n, nvec, base, out, s);
    }
  }
  if (numel > nvec * 4)
    hipLaunchKernelGGL((wsum_f32_arg_tail_kernel<O>), dim3(1), dim3(kTailBlock), 0,
                       s, tab, pre ? 1 : 0, n, nvec * 4, numel, base, out);
}

// ---------------------------------------------------------------------------
// row sets: clients' key tensors read in place (include/fsagg.h fsagg_rows)
// ---------------------------------------------------------------------------
// One chunk of <= kBlock·V float4 coordinates of one key segment.  The
// chunk's client rows are wave-uniform scalar loads of the pointer table; a
// NULL entry is a client that lacks the key and is skipped (the reference's
// `if key not in local_model: continue`, clients_avg_aggregator.py:74-75) —
// the first present client initialises the accumulator.  Same per-lane
// streaming shape as wsum_tile: all V loads of one client in flight before
// any is consumed.
template <int V, bool PRE, bool BASE, bool GUARD>
__device__ __forceinline__ void wsum_rows_chunk(
    const float *const *__restrict__ rows, int n, int64_t lo,
    int nvec, const float *__restrict__ w, const float *__restrict__ pre,
    const float *__restrict__ base, float *__restrict__ out) {
  int idx[V];
  bool ok[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    idx[v] = v * kBlock + int(threadIdx.x);
    ok[v] = !GUARD || idx[v] < nvec;
  }
  // the first present client initialises the accumulator
  int i0 = 0;
  while (i0 < n && rows[i0] == nullptr) ++i0;
  f4 acc[V];
  const uint32_t loff = uint32_t(threadIdx.x) * 16u;   // lane byte offset
  const int cbytes = nvec * 16;                        // the chunk's f4s
  if (i0 < n) {
    const __amdgpu_buffer_rsrc_t r = row_rsrc(rows[i0] + lo, cbytes);
    const float w0 = w[i0];
    const float s0 = PRE ? pre[i0] : 1.0f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      f4 x = ld4_rowv<GUARD>(r, loff, v);
      if (PRE) x = mul4(x, s0);
      acc[v] = mul4(x, w0);
    }
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  }
  // the other clients two at a time, the next one's loads in flight while
  // the current one is added (ping-pong buffers, V <= 16; an absent client
  // loads and adds nothing).  One client in flight measured 0.8–1.1 % slower at
  // the ResNet-50 layout (tools/probe_layout_b.py): the row
  // pointer and buffer descriptor of each client are scalar work the
  // wave otherwise waits behind.
  auto load = [&](f4 (&x)[V], int c) {
    const float *row = rows[c];
    if (row == nullptr) return;
    const __amdgpu_buffer_rsrc_t r = row_rsrc(row + lo, cbytes);
#pragma unroll
    for (int v = 0; v < V; ++v) x[v] = ld4_rowv<GUARD>(r, loff, v);
  };
  auto add = [&](const f4 (&x)[V], int c) {
    if (rows[c] == nullptr) return;
    const float wc = w[c];
    const float sc = PRE ? pre[c] : 1.0f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      f4 t = x[v];
      if (PRE) t = mul4(t, sc);
      acc[v] = add4(acc[v], mul4(t, wc));
    }
  };
  if constexpr (V <= 16) {
    f4 xa[V], xb[V];
    int i = i0 + 1;
    if (i < n) load(xa, i);
    for (; i + 1 < n; i += 2) {
      load(xb, i + 1);
      add(xa, i);
      if (i + 2 < n) load(xa, i + 2);
      add(xb, i + 1);
    }
    if (i < n) add(xa, i);
  } else {
    // V = 24: two buffers would not fit 256 VGPRs
    for (int i = i0 + 1; i < n; ++i) {
      f4 x[V];
      load(x, i);
      add(x, i);
    }
  }
  f4 *o = reinterpret_cast<f4 *>(out + lo);
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (!ok[v]) continue;
    f4 a = acc[v];
    if (BASE) a = add4(ld4<false>(reinterpret_cast<const f4 *>(base + lo) +
                                  idx[v]), a);
    o[idx[v]] = a;
  }
}

template <int V, bool PRE, bool BASE>
__device__ __forceinline__ void wsum_rows_body(
    const float *const *__restrict__ tab, int64_t ss, int n,
    const fsagg_chunk *__restrict__ chunks, int nchunk,
    const float *__restrict__ w, const float *__restrict__ pre,
    const float *const *__restrict__ btab, int64_t bss,
    float *__restrict__ out) {
  for (int c = blockIdx.x; c < nchunk; c += gridDim.x) {
    const int64_t lo = chunks[c].lo;
    const int len = chunks[c].len;
    const int seg = chunks[c].seg;
    const float *const *rows = tab + int64_t(seg) * ss;
    const float *base = BASE ? btab[int64_t(seg) * bss] : nullptr;
    const int nvec = len >> 2;
    if (nvec == kBlock * V)
      wsum_rows_chunk<V, PRE, BASE, false>(rows, n, lo, nvec, w, pre, base,
                                           out);
    else
      wsum_rows_chunk<V, PRE, BASE, true>(rows, n, lo, nvec, w, pre, base,
                                          out);
    // the key's last (< 4) coordinates
    const int t = int(threadIdx.x);
    if (t < (len & 3)) {
      const int64_t p = lo + 4 * int64_t(nvec) + t;
      float acc = 0.0f;
      bool first = true;
      for (int i = 0; i < n; ++i) {
        const float *row = rows[i];
        if (row == nullptr) continue;
        float x = gld(row + p);
        if (PRE) x = mul_rn(x, pre[i]);
        acc = first ? mul_rn(x, w[i]) : add_rn(acc, mul_rn(x, w[i]));
        first = false;
      }
      if (BASE) acc = add_rn(gld(base + p), acc);
      out[p] = acc;
    }
  }
}

template <int V, bool PRE, bool BASE>
__global__ __launch_bounds__(kBlock) void wsum_rows_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n,
    const fsagg_chunk *__restrict__ chunks, int nchunk,
    const float *__restrict__ w, const float *__restrict__ pre,
    const float *const *__restrict__ btab, int64_t bss,
    float *__restrict__ out) {
  wsum_rows_body<V, PRE, BASE>(tab, ss, n, chunks, nchunk, w, pre, btab, bss,
                               out);
}

// The row set's pointer table [nseg][n], weights, prescales and base table
// in the kernel arguments (fsagg_weighted_sum_rows_hosttab_f32): small row
// sets — a multi-Krum selection's average, a handful of clients of a
// multi-key model — whose per-call uploads cost more host time than the
// kernel (each H2D copy ~19 us, profiles/r06/upload_cost.json).
static_assert(FSAGG_HOSTTAB_ROWS_MAX_CLIENTS <= FSAGG_HOSTTAB_ROWS_MAX_PTRS,
              "row-set host table limits");
struct ArgRows {
  const float *tab[FSAGG_HOSTTAB_ROWS_MAX_PTRS];
  const float *base[FSAGG_HOSTTAB_ROWS_MAX_SEGS];
  float w[FSAGG_HOSTTAB_ROWS_MAX_CLIENTS];
  float pre[FSAGG_HOSTTAB_ROWS_MAX_CLIENTS];
};

template <int V, bool PRE, bool BASE>
__global__ __launch_bounds__(kBlock) void wsum_rows_arg_kernel(
    const ArgRows a, int n, const fsagg_chunk *__restrict__ chunks,
    int nchunk, float *__restrict__ out) {
  wsum_rows_body<V, PRE, BASE>(a.tab, n, n, chunks, nchunk, a.w, a.pre,
                               a.base, 1, out);
}

template <int V>
void launch_wsum_rows_arg(const ArgRows &a, bool pre, bool base, int n,
                          const fsagg_chunk *chunks, int nchunk, float *out,
                          hipStream_t s) {
  const unsigned grid = stream_grid(nchunk, 1, 256 * 16);
#define FSAGG_RA(P, B)                                                      \
  hipLaunchKernelGGL((wsum_rows_arg_kernel<V, P, B>), dim3(grid),          \
                     dim3(kBlock), 0, s, a, n, chunks, nchunk, out)
  if (pre) {
    if (base) FSAGG_RA(true, true);
    else FSAGG_RA(true, false);
  } else {
    if (base) FSAGG_RA(false, true);
    else FSAGG_RA(false, false);
  }
#undef FSAGG_RA
}

// V of the row-set kernel's chunks for a bucket of `numel` coordinates of n
// clients (fsagg_wsum_chunk_elems)
// A/B: a fixed row-set chunk width (fsagg_wsum_set_rows_width; 0 = the rule)
std::atomic<int> g_rows_width{0};

int wsum_vec_width(int64_t numel, int n) {
  const int v = g_rows_width.load(std::memory_order_relaxed);
  return v > 0 ? v : wsum_width_rows(numel / 4, n);
}

template <int V, bool PRE, bool BASE>
void launch_wsum_rows(const fsagg_rows &rs, const fsagg_chunk *chunks,
                      int nchunk, const float *w, const float *pre,
                      const float *const *btab, int64_t bss, float *out,
                      hipStream_t s) {
  const unsigned grid = stream_grid(nchunk, 1, 256 * 16);
  hipLaunchKernelGGL((wsum_rows_kernel<V, PRE, BASE>), dim3(grid),
                     dim3(kBlock), 0, s, rs.tab, rs.ss, rs.n, chunks,
                     nchunk, w, pre, btab, bss, out);
}

template <int V>
void launch_wsum_rows_v(const fsagg_rows &rs, const fsagg_chunk *chunks,
                        int nchunk, const float *w, const float *pre,
                        const float *const *btab, int64_t bss, float *out,
                        hipStream_t s) {
  if (pre) {
    if (btab) launch_wsum_rows<V, true, true>(rs, chunks, nchunk, w, pre, btab, bss, out, s);
    else launch_wsum_rows<V, true, false>(rs, chunks, nchunk, w, pre, btab, bss, out, s);
  } else {
    if (btab) launch_wsum_rows<V, false, true>(rs, chunks, nchunk, w, pre, btab, bss, out, s);
    else launch_wsum_rows<V, false, false>(rs, chunks, nchunk, w, pre, btab, bss, out, s);
  }
}

// ---------------------------------------------------------------------------
// non-fp32 buckets
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint16_t f2bf_rne(float f) {
  // c10::detail::round_to_nearest_even
  if (__builtin_isnan(f)) return 0x7FC0;
  uint32_t u = __float_as_uint(f);
  u += ((u >> 16) & 1u) + 0x7FFFu;
  return static_cast<uint16_t>(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(uint32_t(b) << 16);
}

// ATen rounds x*w to float first and then to half (two roundings).  Left
// alone, the backend fuses fptrunc(fmul) into one v_fma_mixlo_f16 (a single
// rounding of the exact product), which differs in the last bit; the empty
// asm makes the fp32 product a materialised value.
__device__ __forceinline__ float mul_f32_materialized(float a, float b) {
  float p = mul_rn(a, b);
  asm volatile("" : "+v"(p));
  return p;
}

template <int DT>
__global__ __launch_bounds__(kBlock) void wsum_typed_kernel(
    const void *const *__restrict__ rows, const double *__restrict__ w, int n,
    int64_t numel, void *__restrict__ out) {
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    if constexpr (DT == FSAGG_F64) {
      double acc = __dmul_rn(gld(static_cast<const double *>(rows[0]) + p), w[0]);
      for (int i = 1; i < n; ++i)
        acc = __dadd_rn(acc,
                        __dmul_rn(gld(static_cast<const double *>(rows[i]) + p), w[i]));
      static_cast<double *>(out)[p] = acc;
    } else if constexpr (DT == FSAGG_F16) {
      auto ld = [&](int i) {
        return __half2float(__ushort_as_half(gld(static_cast<const unsigned short *>(rows[i]) + p)));
      };
      __half acc = __float2half(mul_f32_materialized(ld(0), float(w[0])));
      for (int i = 1; i < n; ++i) {
        __half t = __float2half(mul_f32_materialized(ld(i), float(w[i])));
        acc = __float2half(add_rn(__half2float(acc), __half2float(t)));
      }
      static_cast<__half *>(out)[p] = acc;
    } else if constexpr (DT == FSAGG_BF16) {
      auto ld = [&](int i) {
        return bf2f(gld(static_cast<const uint16_t *>(rows[i]) + p));
      };
      uint16_t acc = f2bf_rne(mul_rn(ld(0), float(w[0])));
      for (int i = 1; i < n; ++i) {
        uint16_t t = f2bf_rne(mul_rn(ld(i), float(w[i])));
        acc = f2bf_rne(add_rn(bf2f(acc), bf2f(t)));
      }
      static_cast<uint16_t *>(out)[p] = acc;
    } else {  // FSAGG_I64 -> f32
      auto ld = [&](int i) {
        return static_cast<float>(gld(static_cast<const int64_t *>(rows[i]) + p));
      };
      float acc = mul_rn(ld(0), float(w[0]));
      for (int i = 1; i < n; ++i) acc = add_rn(acc, mul_rn(ld(i), float(w[i])));
      static_cast<float *>(out)[p] = acc;
    }
  }
}

// ---------------------------------------------------------------------------
// online running mean, init+update add, synthetic fill
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void online_inc_kernel(
    float *__restrict__ m, const float *__restrict__ x, float c, float s,
    float d, int64_t numel) {
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    m[p] = __fdiv_rn(add_rn(mul_rn(c, m[p]), mul_rn(s, x[p])), d);
  }
}

// Online running mean with ATen's dtype rules (clients_avg_aggregator.py:
// 136-139 on tensors of any of f32/f16/bf16/f64/i64): a = cnt*m in m's
// type, b = s*x in x's type (reduced floats computed in float and rounded
// once — ATen's opmath), c = a + b in the promoted type (both operands cast
// to it first), out = c / (cnt + s) — integers become float32 (true
// division).  Values travel as doubles (exact for every float type) or
// int64.  A per-element type switch: this path carries the odd keys (BN
// counters, fp16 uploads), never the bulk.
struct TV {
  double f;
  int64_t i;
};

__device__ __forceinline__ TV load_tv(const void *p, int dt, int64_t k) {
  TV v{0.0, 0};
  switch (dt) {
    case FSAGG_F32: v.f = gld(static_cast<const float *>(p) + k); break;
    case FSAGG_F64: v.f = gld(static_cast<const double *>(p) + k); break;
    case FSAGG_F16:
      v.f = __half2float(__ushort_as_half(
          gld(static_cast<const unsigned short *>(p) + k)));
      break;
    case FSAGG_BF16: v.f = bf2f(gld(static_cast<const uint16_t *>(p) + k)); break;
    default: v.i = gld(static_cast<const int64_t *>(p) + k); break;
  }
  return v;
}

// round a float-computed value to type dt (dt a float type)
__device__ __forceinline__ double round_to(float x, int dt) {
  if (dt == FSAGG_F16) return __half2float(__float2half(x));
  if (dt == FSAGG_BF16) return bf2f(f2bf_rne(x));
  return x;
}

// convert a value of type `from` to type `to` (to a float type)
__device__ __forceinline__ double cast_to(TV v, int from, int to) {
  if (to == FSAGG_F64) return from == FSAGG_I64 ? double(v.i) : v.f;
  const float x = from == FSAGG_I64 ? float(v.i) : float(v.f);
  return round_to(x, to);
}

// python int k * tensor value of type dt
__device__ __forceinline__ TV mul_scalar(TV v, int64_t k, int dt) {
  TV r{0.0, 0};
  if (dt == FSAGG_I64) {
    r.i = int64_t(uint64_t(v.i) * uint64_t(k));
  } else if (dt == FSAGG_F64) {
    r.f = __dmul_rn(v.f, double(k));
  } else {
    r.f = round_to(mul_rn(float(v.f), float(k)), dt);
  }
  return r;
}

__global__ __launch_bounds__(kBlock) void online_typed_kernel(
    const void *__restrict__ m, int mdt, const void *__restrict__ x, int xdt,
    void *__restrict__ out, int cdt, int64_t cnt, int64_t s, int64_t numel) {
  const int odt = cdt == FSAGG_I64 ? FSAGG_F32 : cdt;
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const TV a = mul_scalar(load_tv(m, mdt, p), cnt, mdt);
    const TV b = mul_scalar(load_tv(x, xdt, p), s, xdt);
    double r;
    if (cdt == FSAGG_I64) {
      const int64_t c = int64_t(uint64_t(a.i) + uint64_t(b.i));
      r = __fdiv_rn(float(c), float(cnt + s));
    } else if (cdt == FSAGG_F64) {
      r = __ddiv_rn(__dadd_rn(cast_to(a, mdt, cdt), cast_to(b, xdt, cdt)),
                    double(cnt + s));
    } else {
      const float c = float(round_to(
          add_rn(float(cast_to(a, mdt, cdt)), float(cast_to(b, xdt, cdt))),
          cdt));
      r = round_to(__fdiv_rn(c, float(cnt + s)), cdt);
    }
    switch (odt) {
      case FSAGG_F32: static_cast<float *>(out)[p] = float(r); break;
      case FSAGG_F64: static_cast<double *>(out)[p] = r; break;
      case FSAGG_F16:
        static_cast<__half *>(out)[p] = __float2half(float(r));
        break;
      default: static_cast<uint16_t *>(out)[p] = f2bf_rne(float(r)); break;
    }
  }
}

__global__ __launch_bounds__(kBlock) void add_kernel(
    const float *__restrict__ a, const float *__restrict__ b,
    float *__restrict__ out, int64_t nvec, int64_t numel) {
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x; q < nvec;
       q += stride) {
    f4 x = reinterpret_cast<const f4 *>(a)[q];
    f4 y = reinterpret_cast<const f4 *>(b)[q];
    reinterpret_cast<f4 *>(out)[q] = add4(x, y);
  }
  for (int64_t p = nvec * 4 + int64_t(blockIdx.x) * kBlock + threadIdx.x;
       p < numel; p += stride)
    out[p] = add_rn(a[p], b[p]);
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

__global__ __launch_bounds__(kBlock) void fill_uniform_kernel(
    float *__restrict__ X, int n, int64_t numel, int64_t ld, uint64_t seed,
    int64_t off) {
  const uint64_t total = uint64_t(n) * uint64_t(ld);
  for (uint64_t q = uint64_t(blockIdx.x) * kBlock + threadIdx.x; q < total;
       q += uint64_t(gridDim.x) * kBlock) {
    const uint64_t c = q / uint64_t(ld);
    const uint64_t j = q - c * uint64_t(ld);
    float v = 0.0f;
    if (j < uint64_t(numel)) {
      const uint64_t z = mix64(seed * 0x9E3779B97F4A7C15ull ^ (c << 40) ^
                               (uint64_t(off) + j));
      v = float(uint32_t(z >> 40)) * 0x1p-23f - 1.0f;  // exact, in [-1, 1)
    }
    X[q] = v;
  }
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_weighted_sum_f32(const float *const *rows,
                                      const float *weights,
                                      const float *prescale, int n,
                                      int64_t numel, const float *base,
                                      float *out, fsagg_stream_t stream) {
  if (!rows || !weights || !out || n < 1 || numel < 0) {
    set_error("fsagg_weighted_sum_f32: invalid argument (n=%d numel=%lld)", n,
              (long long)numel);
    return FSAGG_EINVAL;
  }
  if (!aligned16(out) || (base && !aligned16(base))) {
    set_error("fsagg_weighted_sum_f32: out/base must be 16-byte aligned");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  launch_wsum_any(rows, weights, prescale, n, numel, base, out,
                  as_stream(stream));
  return check_launch("fsagg_weighted_sum_f32");
}

extern "C" int fsagg_weighted_sum_bcast_f32(const float *const *rows,
                                            const float *weights,
                                            const float *prescale, int n,
                                            int64_t numel, const float *base,
                                            float *const *outs, int nout,
                                            fsagg_stream_t stream) {
  if (!rows || !weights || !outs || n < 1 || numel < 0 || nout < 1 ||
      nout > FSAGG_MAX_PEERS) {
    set_error("fsagg_weighted_sum_bcast_f32: invalid argument (n=%d "
              "numel=%lld nout=%d)", n, (long long)numel, nout);
    return FSAGG_EINVAL;
  }
  Bcast o{};
  o.n = nout;
  for (int k = 0; k < nout; ++k) {
    if (!outs[k] || !aligned16(outs[k])) {
      set_error("fsagg_weighted_sum_bcast_f32: out %d is NULL or not "
                "16-byte aligned", k);
      return FSAGG_EINVAL;
    }
    o.p[k] = outs[k];
  }
  if (base && !aligned16(base)) {
    set_error("fsagg_weighted_sum_bcast_f32: base must be 16-byte aligned");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  launch_wsum_any(rows, weights, prescale, n, numel, base, o,
                  as_stream(stream));
  return check_launch("fsagg_weighted_sum_bcast_f32");
}

extern "C" int fsagg_weighted_sum_hosttab_f32(
    const uint64_t *rows, const float *weights, const float *prescale, int n,
    int64_t numel, const float *base, float *const *outs, int nout,
    fsagg_stream_t stream) {
  if (!rows || !weights || !outs || n < 1 ||
      n > FSAGG_HOSTTAB_MAX_CLIENTS || numel < 0 || nout < 1 ||
      nout > FSAGG_MAX_PEERS) {
    set_error("fsagg_weighted_sum_hosttab_f32: invalid argument (n=%d, at "
              "most %d; numel=%lld nout=%d)", n, FSAGG_HOSTTAB_MAX_CLIENTS,
              (long long)numel, nout);
    return FSAGG_EINVAL;
  }
  ArgTab tab;
  for (int i = 0; i < n; ++i) {
    tab.rows[i] = reinterpret_cast<const float *>(rows[i]);
    if (!tab.rows[i] || !aligned16(tab.rows[i])) {
      set_error("fsagg_weighted_sum_hosttab_f32: row %d is NULL or not "
                "16-byte aligned", i);
      return FSAGG_EINVAL;
    }
    tab.w[i] = weights[i];
    tab.pre[i] = prescale ? prescale[i] : 1.0f;
  }
  for (int i = n; i < FSAGG_HOSTTAB_MAX_CLIENTS; ++i) {
    tab.rows[i] = nullptr;
    tab.w[i] = tab.pre[i] = 0.0f;
  }
  for (int k = 0; k < nout; ++k)
    if (!outs[k] || !aligned16(outs[k])) {
      set_error("fsagg_weighted_sum_hosttab_f32: out %d is NULL or not "
                "16-byte aligned", k);
      return FSAGG_EINVAL;
    }
  if (base && !aligned16(base)) {
    set_error("fsagg_weighted_sum_hosttab_f32: base must be 16-byte "
              "aligned");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  hipStream_t s = as_stream(stream);
  if (nout == 1) {
    launch_wsum_arg_any(tab, prescale != nullptr, n, numel, base, outs[0], s);
  } else {
    Bcast o{};
    o.n = nout;
    for (int k = 0; k < nout; ++k) o.p[k] = outs[k];
    launch_wsum_arg_any(tab, prescale != nullptr, n, numel, base, o, s);
  }
  return check_launch("fsagg_weighted_sum_hosttab_f32");
}

extern "C" int fsagg_wsum_set_rows_width(int v) {
  const int w = v == 24 || v == 16 || v == 8 || v == 4 || v == 1 ? v : 0;
  return fsagg::g_rows_width.exchange(w);
}

extern "C" int64_t fsagg_wsum_chunk_elems(int64_t numel) {
  return int64_t(1024) * wsum_vec_width(numel < 0 ? 0 : numel, 0);
}

extern "C" int64_t fsagg_wsum_chunk_elems_n(int64_t numel, int n) {
  return int64_t(1024) * wsum_vec_width(numel < 0 ? 0 : numel, n);
}

extern "C" int fsagg_weighted_sum_rows_f32(const fsagg_rows *rows,
                                           const fsagg_chunk *chunks,
                                           int nchunk, int64_t chunk_elems,
                                           const float *weights,
                                           const float *prescale,
                                           const float *const *base,
                                           int64_t base_ss, float *out,
                                           fsagg_stream_t stream) {
  if (!rows || !rows->tab || rows->n < 1 || rows->nseg < 1 || !weights ||
      !out || nchunk < 0 || (nchunk > 0 && !chunks) || base_ss < 0) {
    set_error("fsagg_weighted_sum_rows_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (!aligned16(out)) {
    set_error("fsagg_weighted_sum_rows_f32: out must be 16-byte aligned");
    return FSAGG_EINVAL;
  }
  if (nchunk == 0) return FSAGG_OK;
  hipStream_t s = as_stream(stream);
  switch (chunk_elems) {
    case 1024 * 24: launch_wsum_rows_v<24>(*rows, chunks, nchunk, weights, prescale, base, base_ss, out, s); break;
    case 1024 * 16: launch_wsum_rows_v<16>(*rows, chunks, nchunk, weights, prescale, base, base_ss, out, s); break;
    case 1024 * 8: launch_wsum_rows_v<8>(*rows, chunks, nchunk, weights, prescale, base, base_ss, out, s); break;
    case 1024 * 4: launch_wsum_rows_v<4>(*rows, chunks, nchunk, weights, prescale, base, base_ss, out, s); break;
    case 1024: launch_wsum_rows_v<1>(*rows, chunks, nchunk, weights, prescale, base, base_ss, out, s); break;
    default:
      set_error("fsagg_weighted_sum_rows_f32: chunk_elems %lld is not a "
                "fsagg_wsum_chunk_elems() unit", (long long)chunk_elems);
      return FSAGG_EINVAL;
  }
  return check_launch("fsagg_weighted_sum_rows_f32");
}

extern "C" int fsagg_weighted_sum_rows_hosttab_f32(
    const uint64_t *tab, int n, int nseg, const fsagg_chunk *chunks,
    int nchunk, int64_t chunk_elems, const float *weights,
    const float *prescale, const uint64_t *base, float *out,
    fsagg_stream_t stream) {
  if (!tab || n < 1 || n > FSAGG_HOSTTAB_ROWS_MAX_CLIENTS || nseg < 1 ||
      int64_t(n) * nseg > FSAGG_HOSTTAB_ROWS_MAX_PTRS ||
      (base && nseg > FSAGG_HOSTTAB_ROWS_MAX_SEGS) || !weights || !out ||
      nchunk < 0 || (nchunk > 0 && !chunks)) {
    set_error("fsagg_weighted_sum_rows_hosttab_f32: invalid argument (n=%d "
              "nseg=%d; at most %d clients, %d pointers, %d base keys)", n,
              nseg, FSAGG_HOSTTAB_ROWS_MAX_CLIENTS,
              FSAGG_HOSTTAB_ROWS_MAX_PTRS, FSAGG_HOSTTAB_ROWS_MAX_SEGS);
    return FSAGG_EINVAL;
  }
  if (!aligned16(out)) {
    set_error("fsagg_weighted_sum_rows_hosttab_f32: out must be 16-byte "
              "aligned");
    return FSAGG_EINVAL;
  }
  if (nchunk == 0) return FSAGG_OK;
  ArgRows a;
  for (int i = 0; i < n * nseg; ++i)
    a.tab[i] = reinterpret_cast<const float *>(uintptr_t(tab[i]));
  for (int i = n * nseg; i < FSAGG_HOSTTAB_ROWS_MAX_PTRS; ++i)
    a.tab[i] = nullptr;
  for (int k = 0; k < FSAGG_HOSTTAB_ROWS_MAX_SEGS; ++k)
    a.base[k] = base && k < nseg
                    ? reinterpret_cast<const float *>(uintptr_t(base[k]))
                    : nullptr;
  for (int i = 0; i < FSAGG_HOSTTAB_ROWS_MAX_CLIENTS; ++i) {
    a.w[i] = i < n ? weights[i] : 0.0f;
    a.pre[i] = i < n && prescale ? prescale[i] : 1.0f;
  }
  hipStream_t s = as_stream(stream);
  const bool pre = prescale != nullptr, b = base != nullptr;
  switch (chunk_elems) {
    case 1024 * 24: launch_wsum_rows_arg<24>(a, pre, b, n, chunks, nchunk, out, s); break;
    case 1024 * 16: launch_wsum_rows_arg<16>(a, pre, b, n, chunks, nchunk, out, s); break;
    case 1024 * 8: launch_wsum_rows_arg<8>(a, pre, b, n, chunks, nchunk, out, s); break;
    case 1024 * 4: launch_wsum_rows_arg<4>(a, pre, b, n, chunks, nchunk, out, s); break;
    case 1024: launch_wsum_rows_arg<1>(a, pre, b, n, chunks, nchunk, out, s); break;
    default:
      set_error("fsagg_weighted_sum_rows_hosttab_f32: chunk_elems %lld is "
                "not a fsagg_wsum_chunk_elems() unit",
                (long long)chunk_elems);
      return FSAGG_EINVAL;
  }
  return check_launch("fsagg_weighted_sum_rows_hosttab_f32");
}

extern "C" int fsagg_weighted_sum_typed(const void *const *rows, int in_dtype,
                                        const double *weights, int n,
                                        int64_t numel, void *out,
                                        fsagg_stream_t stream) {
  if (!rows || !weights || !out || n < 1 || numel < 0) {
    set_error("fsagg_weighted_sum_typed: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  hipStream_t s = as_stream(stream);
  const unsigned grid = stream_grid(numel, kBlock, 256 * 8);
  switch (in_dtype) {
    case FSAGG_F16:
      hipLaunchKernelGGL(wsum_typed_kernel<FSAGG_F16>, dim3(grid), dim3(kBlock), 0, s, rows, weights, n, numel, out);
      break;
    case FSAGG_BF16:
      hipLaunchKernelGGL(wsum_typed_kernel<FSAGG_BF16>, dim3(grid), dim3(kBlock), 0, s, rows, weights, n, numel, out);
      break;
    case FSAGG_F64:
      hipLaunchKernelGGL(wsum_typed_kernel<FSAGG_F64>, dim3(grid), dim3(kBlock), 0, s, rows, weights, n, numel, out);
      break;
    case FSAGG_I64:
      hipLaunchKernelGGL(wsum_typed_kernel<FSAGG_I64>, dim3(grid), dim3(kBlock), 0, s, rows, weights, n, numel, out);
      break;
    default:
      set_error("fsagg_weighted_sum_typed: unsupported dtype %d", in_dtype);
      return FSAGG_EINVAL;
  }
  return check_launch("fsagg_weighted_sum_typed");
}

extern "C" int fsagg_online_inc_f32(float *m, const float *x, float cnt,
                                    float s, float denom, int64_t numel,
                                    fsagg_stream_t stream) {
  if (!m || !x || numel < 0) {
    set_error("fsagg_online_inc_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  hipLaunchKernelGGL(online_inc_kernel, dim3(stream_grid(numel, kBlock, 256 * 8)),
                     dim3(kBlock), 0, as_stream(stream), m, x, cnt, s, denom,
                     numel);
  return check_launch("fsagg_online_inc_f32");
}

extern "C" int fsagg_online_inc_typed(const void *m, int m_dtype,
                                      const void *x, int x_dtype, void *out,
                                      int common_dtype, int64_t cnt,
                                      int64_t s, int64_t numel,
                                      fsagg_stream_t stream) {
  auto ok = [](int d) { return d >= FSAGG_F32 && d <= FSAGG_I64; };
  if (!m || !x || !out || numel < 0 || !ok(m_dtype) || !ok(x_dtype) ||
      !ok(common_dtype)) {
    set_error("fsagg_online_inc_typed: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  hipLaunchKernelGGL(online_typed_kernel,
                     dim3(stream_grid(numel, kBlock, 256 * 8)), dim3(kBlock),
                     0, as_stream(stream), m, m_dtype, x, x_dtype, out,
                     common_dtype, cnt, s, numel);
  return check_launch("fsagg_online_inc_typed");
}

extern "C" int fsagg_add_f32(const float *a, const float *b, float *out,
                             int64_t numel, fsagg_stream_t stream) {
  if (!a || !b || !out || numel < 0) {
    set_error("fsagg_add_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (!aligned16(a) || !aligned16(b) || !aligned16(out)) {
    set_error("fsagg_add_f32: pointers must be 16-byte aligned");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  const int64_t nvec = numel / 4;
  hipLaunchKernelGGL(add_kernel, dim3(stream_grid(nvec + 1, kBlock, 256 * 8)),
                     dim3(kBlock), 0, as_stream(stream), a, b, out, nvec, numel);
  return check_launch("fsagg_add_f32");
}

extern "C" int fsagg_fill_uniform_f32(float *X, int n, int64_t numel,
                                      int64_t ld, uint64_t seed,
                                      int64_t index_offset,
                                      fsagg_stream_t stream) {
  if (!X || n < 1 || numel < 0 || ld < numel) {
    set_error("fsagg_fill_uniform_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  const int64_t total = int64_t(n) * ld;
  if (total == 0) return FSAGG_OK;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(stream_grid(total, kBlock, 256 * 16)),
                     dim3(kBlock), 0, as_stream(stream), X, n, numel, ld, seed,
                     index_offset);
  return check_launch("fsagg_fill_uniform_f32");
}

// ---------------------------------------------------------------------------
// Internal tuning entry points (tools/tune_wsum.py); not part of the ABI.
// ---------------------------------------------------------------------------
namespace fsagg {
namespace {

template <int U, int V, bool NT>
void launch_variant(const float *const *rows, const float *w, int n,
                    int64_t nvec, float *out, unsigned grid, hipStream_t s) {
  const int64_t tiles = (nvec + int64_t(kBlock) * V - 1) / (int64_t(kBlock) * V);
  if (grid == 0) grid = stream_grid(tiles, 1, 256 * 16);
  hipLaunchKernelGGL((wsum_f32_vec_kernel<U, V, false, false, NT>),
                     dim3(grid), dim3(kBlock), 0, s, rows, w, nullptr, n, nvec,
                     nullptr, out);
}

// read-only stream: Σ of a buffer per thread, one float written per thread
template <bool NT>
__global__ __launch_bounds__(kBlock) void readbw_kernel(const f4 *__restrict__ x,
                                                        int64_t nvec,
                                                        float *__restrict__ out) {
  f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  for (; q + 3 * stride < nvec; q += 4 * stride) {
    const f4 a = ld4<NT>(x + q), b = ld4<NT>(x + q + stride),
             c = ld4<NT>(x + q + 2 * stride), d = ld4<NT>(x + q + 3 * stride);
    acc += a + b + c + d;
  }
  for (; q < nvec; q += stride) acc += ld4<NT>(x + q);
  out[int64_t(blockIdx.x) * kBlock + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

}  // namespace
}  // namespace fsagg

extern "C" int fsagg_tune_wsum(int variant, unsigned grid,
                               const float *const *rows, const float *w, int n,
                               int64_t numel, float *out,
                               fsagg_stream_t stream) {
  using namespace fsagg;
  hipStream_t s = as_stream(stream);
  const int64_t nvec = numel / 4;
  switch (variant) {
    case 0: launch_variant<8, 2, true>(rows, w, n, nvec, out, grid, s); break;
    case 1: launch_variant<2, 8, true>(rows, w, n, nvec, out, grid, s); break;
    case 2: launch_variant<4, 8, true>(rows, w, n, nvec, out, grid, s); break;
    case 3: launch_variant<1, 8, true>(rows, w, n, nvec, out, grid, s); break;
    case 4: launch_variant<2, 16, true>(rows, w, n, nvec, out, grid, s); break;
    case 5: launch_variant<1, 16, true>(rows, w, n, nvec, out, grid, s); break;
    case 6: launch_variant<4, 4, true>(rows, w, n, nvec, out, grid, s); break;
    case 7: launch_variant<3, 8, true>(rows, w, n, nvec, out, grid, s); break;
    case 8: launch_variant<2, 8, false>(rows, w, n, nvec, out, grid, s); break;
    case 9: launch_variant<1, 12, true>(rows, w, n, nvec, out, grid, s); break;
    case 10: launch_variant<1, 20, true>(rows, w, n, nvec, out, grid, s); break;
    case 11: launch_variant<1, 24, true>(rows, w, n, nvec, out, grid, s); break;
    case 12: launch_variant<1, 1, true>(rows, w, n, nvec, out, grid, s); break;
    case 13: launch_variant<4, 1, true>(rows, w, n, nvec, out, grid, s); break;
    case 14: launch_variant<8, 1, true>(rows, w, n, nvec, out, grid, s); break;
    case 15: launch_variant<2, 4, true>(rows, w, n, nvec, out, grid, s); break;
    case 16: launch_variant<1, 4, true>(rows, w, n, nvec, out, grid, s); break;
    case 17: launch_variant<4, 2, true>(rows, w, n, nvec, out, grid, s); break;
    default: set_error("variant"); return FSAGG_EINVAL;
  }
  return check_launch("fsagg_tune_wsum");
}

extern "C" int fsagg_tune_wsum_part(int variant, unsigned grid,
                                    const float *const *rows, const float *w,
                                    int n, int64_t numel, float *out,
                                    fsagg_stream_t stream) {
  using namespace fsagg;
  hipStream_t s = as_stream(stream);
  const int64_t nvec = numel / 4;
  int64_t chunk = (nvec + grid - 1) / grid;
  chunk = (chunk + 63) / 64 * 64;
#define FSAGG_TP(U, V)                                                        \
  hipLaunchKernelGGL((wsum_f32_part_kernel<U, V, false, false, true>),       \
                     dim3(grid), dim3(kBlock), 0, s, rows, w, nullptr, n,    \
                     nvec, chunk, nullptr, out)
  switch (variant) {
    case 0: FSAGG_TP(1, 8); break;
    case 1: FSAGG_TP(1, 12); break;
    case 2: FSAGG_TP(1, 16); break;
    case 3: FSAGG_TP(1, 24); break;
    case 4: FSAGG_TP(2, 8); break;
    case 5: FSAGG_TP(2, 12); break;
    case 6: FSAGG_TP(1, 32); break;
    case 7: FSAGG_TP(4, 4); break;
    default: set_error("variant"); return FSAGG_EINVAL;
  }
#undef FSAGG_TP
  return check_launch("fsagg_tune_wsum_part");
}

extern "C" int fsagg_tune_readbw(int nt, unsigned grid, const float *x,
                                 int64_t numel, float *out,
                                 fsagg_stream_t stream) {
  using namespace fsagg;
  const int64_t nvec = numel / 4;
  if (nt)
    hipLaunchKernelGGL(readbw_kernel<true>, dim3(grid), dim3(kBlock), 0,
                       as_stream(stream), reinterpret_cast<const f4 *>(x),
                       nvec, out);
  else
    hipLaunchKernelGGL(readbw_kernel<false>, dim3(grid), dim3(kBlock), 0,
                       as_stream(stream), reinterpret_cast<const f4 *>(x),
                       nvec, out);
  return check_launch("fsagg_tune_readbw");
}
