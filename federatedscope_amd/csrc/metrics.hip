// Update-dissimilarity metrics over the client stack (gfx950):
// per-row, per-key Σ (x - base)^2 in fp64, the ‖local − last‖² terms of
// calc_l2_dissim and calc_blocal_dissim
// (federatedscope/core/monitors/metric_calculator.py:309-372).
//
// Work: chunks of ≤ chl coordinates that never straddle a key; block =
// (chunk, row) reduces its chunk in fp64 (wave shuffles, then the 4 waves in
// order) → partial[chunk][row]; a second kernel sums each key's chunks in
// chunk order.  Deterministic, HBM-bound (4 B per element, +4 B of base that
// stays L2-resident across the rows of a chunk).
#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;

struct DeltaPlan {
  int64_t chl;
  int64_t max_chunks;
};

DeltaPlan delta_plan(int64_t numel, int nseg) {
  DeltaPlan pl;
  int64_t chl = (numel + 255) / 256;
  if (chl < 4096) chl = 4096;
  pl.chl = (chl + 255) / 256 * 256;
  pl.max_chunks = numel / pl.chl + nseg + 1;
  return pl;
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

__global__ void delta_prefix_kernel(const int64_t *__restrict__ seg_off,
                                    int nseg, int64_t chl, int *prefix) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int acc = 0;
  prefix[0] = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_off[s + 1] - seg_off[s];
    acc += int((len + chl - 1) / chl);
    prefix[s + 1] = acc;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// Where client `row`'s coordinate `start` (inside key `s`) lives: a flat
// stack row, or (KEYS) the client's own tensor for key s — table entry
// [row][s] of an n x nseg pointer table, so device-resident client dicts
// are read in place instead of being staged into a stack first.
template <bool KEYS>
__device__ __forceinline__ const float *row_at(const float *const *rows,
                                               int row, int nseg, int s,
                                               const int64_t *seg_off,
                                               int64_t p) {
  if (KEYS) return rows[int64_t(row) * nseg + s] + (p - seg_off[s]);
  return rows[row] + p;
}

template <bool KEYS>
__device__ __forceinline__ const float *base_at(const float *base,
                                                const float *const *base_keys,
                                                int s, const int64_t *seg_off,
                                                int64_t p) {
  if (KEYS) return base_keys ? base_keys[s] + (p - seg_off[s]) : nullptr;
  return base ? base + p : nullptr;
}

// One lane's fp64 Σ fl32(x - b)^2 over coordinates lane, lane + kBlock, ...
// of a chunk: unguarded groups of 8 coordinates (all loads issued before
// the first use), then a guarded tail.
template <bool BASE>
__device__ __forceinline__ double chunk_sqsum(const float *__restrict__ x,
                                              const float *__restrict__ b,
                                              int len) {
  constexpr int G = 8;
  const int full = len / (G * kBlock) * (G * kBlock);
  double acc = 0.0;
  int q = threadIdx.x;
  for (; q < full; q += G * kBlock) {
    float v[G], bv[G];
#pragma unroll
    for (int e = 0; e < G; ++e) {
      v[e] = gload_nt(x + q + e * kBlock);
      if (BASE) bv[e] = gload(b + q + e * kBlock);
    }
#pragma unroll
    for (int e = 0; e < G; ++e) {
      const float d = BASE ? __fsub_rn(v[e], bv[e]) : v[e];
      acc += double(d) * double(d);
    }
  }
  for (; q < len; q += kBlock) {
    const float d = BASE ? __fsub_rn(gload(x + q), gload(b + q)) : gload(x + q);
    acc += double(d) * double(d);
  }
  return acc;
}

// Block (chunk c, row): chunk_sqsum per lane (one fp64 accumulator, fixed
// order), then the wave and block sums in order.
template <bool KEYS>
__global__ __launch_bounds__(kBlock) void delta_partial_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ base,
    const float *const *__restrict__ base_keys,
    const int64_t *__restrict__ seg_off, int nseg,
    const int *__restrict__ prefix, int64_t chl, double *__restrict__ partial,
    int n) {
  __shared__ double red[kBlock / kWave];
  // rows fastest: the n blocks of one chunk run together, so the chunk of
  // `base` they all subtract stays in L2 instead of streaming n times
  const int row = blockIdx.x, c = blockIdx.y;
  const int total = prefix[nseg];
  if (c >= total) return;
  int lo = 0, hi = nseg;  // segment: largest s with prefix[s] <= c
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= c) lo = mid;
    else hi = mid;
  }
  const int64_t start = seg_off[lo] + int64_t(c - prefix[lo]) * chl;
  int64_t end = start + chl;
  if (end > seg_off[lo + 1]) end = seg_off[lo + 1];
  const int len = int(end - start);
  const float *x = row_at<KEYS>(rows, row, nseg, lo, seg_off, start);
  const float *b = base_at<KEYS>(base, base_keys, lo, seg_off, start);
  const double acc = b ? chunk_sqsum<true>(x, b, len)
                       : chunk_sqsum<false>(x, nullptr, len);
  const double wsum = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = wsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) t += red[w];
    partial[int64_t(c) * n + row] = t;
  }
}

// sq[row][s] = Σ over segment s's chunks: one wave per (row, s), lanes
// striding the chunks, then the wave sum (a fixed order).
__global__ __launch_bounds__(kBlock) void delta_final_kernel(
    const double *__restrict__ partial, const int *__restrict__ prefix,
    int nseg, int n, double *__restrict__ sq) {
  const int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (q >= int64_t(n) * nseg) return;
  const int row = int(q / nseg), s = int(q % nseg);
  double t = 0.0;
  for (int c = prefix[s] + lane; c < prefix[s + 1]; c += kWave)
    t += partial[int64_t(c) * n + row];
  t = wave_sum(t);
  if (lane == 0) sq[q] = t;
}

// Rows [0, n - n % 8) of the fast path: eight row pointers fetched together
// (scalar loads), then 32 coordinates in flight; GUARD only for the grid's
// last, partial block.  Returns the first row not yet added.
template <bool KEYS, bool GUARD>
__device__ __forceinline__ int wsum_rows(const float *const *__restrict__ rows,
                                         const float *__restrict__ w, int n,
                                         int nseg, int sb, int64_t q0,
                                         const bool (&live)[4],
                                         const float (&b)[4], float (&acc)[4]) {
  constexpr int R = 8;
  int i = 0;
  for (; i + R <= n; i += R) {
    const float *r[R];
#pragma unroll
    for (int u = 0; u < R; ++u)
      r[u] = KEYS ? rows[int64_t(i + u) * nseg + sb] : rows[i + u];
    float x[R][4];
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        x[u][e] = (!GUARD || live[e]) ? gload_nt(r[u] + q0 + e * kBlock)
                                      : 0.0f;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const float wu = w[i + u];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[e] = add_rn(acc[e], mul_rn(wu, __fsub_rn(x[u][e], b[e])));
    }
  }
  return i;
}

// out[p] = Σ_i fl32(w_i * fl32(x_i[p] - base[p])), list order, from +0:
// the global update of calc_blocal_dissim (metric_calculator.py:342-349).
// Four coordinates per lane (stride kBlock) and eight rows per step, so 32
// loads are in flight; each coordinate still adds its rows in order.
template <bool KEYS>
__global__ __launch_bounds__(kBlock) void delta_wsum_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w, int n,
    int64_t numel, const float *__restrict__ base,
    const float *const *__restrict__ base_keys,
    const int64_t *__restrict__ seg_off, int nseg, float *__restrict__ out) {
  const int64_t blk0 = int64_t(blockIdx.x) * 4 * kBlock;
  const int64_t p0 = blk0 + threadIdx.x;
  // KEYS: the key holding the block's first coordinate (a block-uniform,
  // scalar search); when the block's 4*kBlock coordinates all lie in it,
  // every row pointer is one scalar load, as in the flat form.
  int sb = 0;
  bool uniform = true;
  if (KEYS) {
    int lo = 0, hi = nseg;  // largest s with seg_off[s] <= blk0
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg_off[mid] <= blk0) lo = mid;
      else hi = mid;
    }
    sb = lo;
    uniform = seg_off[sb + 1] >= blk0 + 4 * kBlock || seg_off[sb + 1] >= numel;
  }
  if (p0 >= numel) return;
  int64_t p[4];
  int s[4];
  bool live[4];
  int sc = sb;
  float b[4], acc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    p[e] = p0 + int64_t(e) * kBlock;
    live[e] = p[e] < numel;
    if (KEYS && !uniform)
      while (live[e] && p[e] >= seg_off[sc + 1]) ++sc;
    s[e] = sc;
    b[e] = live[e] ? gload(base_at<KEYS>(base, base_keys, s[e], seg_off, p[e]))
                   : 0.0f;
    acc[e] = 0.0f;
  }
  int i = 0;
  if (!KEYS || uniform) {
    const int64_t q0 = p0 - (KEYS ? seg_off[sb] : 0);  // row pointers per key
    if (blk0 + 4 * kBlock <= numel)
      i = wsum_rows<KEYS, false>(rows, w, n, nseg, sb, q0, live, b, acc);
    else
      i = wsum_rows<KEYS, true>(rows, w, n, nseg, sb, q0, live, b, acc);
  }
  // remaining rows (and every row of a block that straddles keys)
  for (; i < n; ++i) {
    const float wi = w[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xv =
          live[e] ? gload(row_at<KEYS>(rows, i, nseg, s[e], seg_off, p[e])) : 0.0f;
      acc[e] = add_rn(acc[e], mul_rn(wi, __fsub_rn(xv, b[e])));
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (live[e]) out[p[e]] = acc[e];
}


// calc_blocal_dissim's two client passes in ONE read of the clients: the
// per-row, per-key Σ fl32(x − b)² of delta_partial_kernel and the weighted
// sum out[p] = Σ_i fl32(w_i · fl32(x_i[p] − b[p])) of delta_wsum_kernel
// (rows in order from +0: `out` is bit-identical to it).  One wave per
// chunk of kFuseChunk coordinates that never straddles a key; lane l holds
// coordinates 4l + 256j (j < 4): 16 base values and 16 wsum accumulators in
// registers.  The wave walks the rows in order: when the chunk is whole
// and every row's piece 16-B aligned, three rows' 16-B non-temporal loads
// stay in flight (fuse_rows_vec); else the next row's loads (16-B where
// that row allows, guarded 4-B otherwise) are issued before the current
// row's arithmetic.  It leaves each row's fp64 chunk sum (the lanes' sums, then the wave sum) in
// partial[chunk][row]; delta_final_kernel adds a key's chunks in order.
constexpr int kFuseChunk = 1024;
constexpr int kFuseE = kFuseChunk / kWave;  // 16 values per lane
typedef float f4x __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int fuse_idx(int lane, int k) {
  return 4 * lane + 256 * (k >> 2) + (k & 3);
}

__device__ __forceinline__ void fuse_load(const float *x, bool vec, int len,
                                          int lane, float (&v)[kFuseE]) {
  if (vec) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f4x q = gld_nt(reinterpret_cast<const f4x *>(x + 4 * lane + 256 * j));
      v[4 * j] = q.x;
      v[4 * j + 1] = q.y;
      v[4 * j + 2] = q.z;
      v[4 * j + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kFuseE; ++k) {
      const int idx = fuse_idx(lane, k);
      v[k] = idx < len ? gload(x + idx) : 0.0f;
    }
  }
}

// One row of the fused pass: d = x − b into the wsum accumulators and the
// row's fp64 sum of squares (wave sum) into part[i].
__device__ __forceinline__ void fuse_row(const float (&xv)[kFuseE],
                                         const float (&bv)[kFuseE], float wi,
                                         float (&acc)[kFuseE], int lane,
                                         double *part) {
  double sq = 0.0;
#pragma unroll
  for (int k = 0; k < kFuseE; ++k) {
    const float d = __fsub_rn(xv[k], bv[k]);
    acc[k] = add_rn(acc[k], mul_rn(wi, d));
    sq = __fma_rn(double(d), double(d), sq);
  }
  sq = wave_sum(sq);
  // lane 0's total, stored by every lane (one address): no exec-masked
  // store whose skip would blur the compiler's load counts
  const uint64_t t = __double_as_longlong(sq);
  const uint32_t tlo = __builtin_amdgcn_readfirstlane(uint32_t(t));
  const uint32_t thi = __builtin_amdgcn_readfirstlane(uint32_t(t >> 32));
  *part = __longlong_as_double(int64_t(uint64_t(tlo) | (uint64_t(thi) << 32)));
}

__device__ __forceinline__ void fuse_vec(const float *x, int lane,
                                         float (&v)[kFuseE]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f4x q = gld_nt(reinterpret_cast<const f4x *>(x + 4 * lane + 256 * j));
    v[4 * j] = q.x;
    v[4 * j + 1] = q.y;
    v[4 * j + 2] = q.z;
    v[4 * j + 3] = q.w;
  }
}

// Whole, aligned chunks: three rows' 16-B loads in flight while a row is
// summed (buffers A, B, C in rotation).
template <bool KEYS>
__device__ __forceinline__ void fuse_rows_vec(
    const float *const *__restrict__ rows, const float *__restrict__ w,
    int n, int nseg, int lo, const int64_t *__restrict__ seg_off,
    int64_t start, int lane, const float (&bv)[kFuseE],
    float (&acc)[kFuseE], double *part) {
  auto rp = [&](int i) {
    return row_at<KEYS>(rows, i, nseg, lo, seg_off, start);
  };
  float xa[kFuseE], xb[kFuseE], xc[kFuseE];
  fuse_vec(rp(0), lane, xa);
  if (n > 1) fuse_vec(rp(1), lane, xb);
  if (n > 2) fuse_vec(rp(2), lane, xc);
  // steady state without branches (the compiler's load counts stay exact:
  // a row's wait leaves the two later rows' loads in flight)
  int i = 0;
  for (; i + 5 < n; i += 3) {
    fuse_row(xa, bv, w[i], acc, lane, part + i);
    fuse_vec(rp(i + 3), lane, xa);
    fuse_row(xb, bv, w[i + 1], acc, lane, part + i + 1);
    fuse_vec(rp(i + 4), lane, xb);
    fuse_row(xc, bv, w[i + 2], acc, lane, part + i + 2);
    fuse_vec(rp(i + 5), lane, xc);
  }
  // the last <= 5 rows: i, i + 1, i + 2 are loaded (those < n)
  if (i < n) fuse_row(xa, bv, w[i], acc, lane, part + i);
  if (i + 3 < n) fuse_vec(rp(i + 3), lane, xa);
  if (i + 1 < n) fuse_row(xb, bv, w[i + 1], acc, lane, part + i + 1);
  if (i + 4 < n) fuse_vec(rp(i + 4), lane, xb);
  if (i + 2 < n) fuse_row(xc, bv, w[i + 2], acc, lane, part + i + 2);
  if (i + 3 < n) fuse_row(xa, bv, w[i + 3], acc, lane, part + i + 3);
  if (i + 4 < n) fuse_row(xb, bv, w[i + 4], acc, lane, part + i + 4);
}

template <bool KEYS>
__global__ __launch_bounds__(kWave) void delta_fused_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w, int n,
    const float *__restrict__ base, const float *const *__restrict__ base_keys,
    const int64_t *__restrict__ seg_off, int nseg,
    const int *__restrict__ prefix, double *__restrict__ partial,
    float *__restrict__ out) {
  const int c = blockIdx.x;
  const int total = prefix[nseg];
  if (c >= total) return;
  int lo = 0, hi = nseg;  // segment: largest s with prefix[s] <= c
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= c) lo = mid;
    else hi = mid;
  }
  const int64_t start = seg_off[lo] + int64_t(c - prefix[lo]) * kFuseChunk;
  int64_t end = start + kFuseChunk;
  if (end > seg_off[lo + 1]) end = seg_off[lo + 1];
  const int len = int(end - start);
  const int lane = threadIdx.x;
  const float *b = base_at<KEYS>(base, base_keys, lo, seg_off, start);
  float bv[kFuseE], acc[kFuseE], xn[kFuseE];
#pragma unroll
  for (int k = 0; k < kFuseE; ++k) {
    const int idx = fuse_idx(lane, k);
    bv[k] = (b && idx < len) ? gload(b + idx) : 0.0f;
    acc[k] = 0.0f;
  }
  const bool whole = len == kFuseChunk;
  // every row's chunk whole and 16-B aligned (the lanes check the rows'
  // pointers, then a ballot): the three-deep pipeline of 16-B loads
  bool odd = false;
  if (whole)
    for (int i = lane; i < n; i += kWave)
      odd |= (reinterpret_cast<uintptr_t>(
                  row_at<KEYS>(rows, i, nseg, lo, seg_off, start)) & 15) != 0;
  if (whole && !__any(odd)) {
    fuse_rows_vec<KEYS>(rows, w, n, nseg, lo, seg_off, start, lane, bv, acc,
                        partial + int64_t(c) * n);
  } else {
  {
    const float *x = row_at<KEYS>(rows, 0, nseg, lo, seg_off, start);
    fuse_load(x, whole && (reinterpret_cast<uintptr_t>(x) & 15) == 0, len,
              lane, xn);
  }
  for (int i = 0; i < n; ++i) {
    float xv[kFuseE];
#pragma unroll
    for (int k = 0; k < kFuseE; ++k) xv[k] = xn[k];
    if (i + 1 < n) {
      const float *x = row_at<KEYS>(rows, i + 1, nseg, lo, seg_off, start);
      fuse_load(x, whole && (reinterpret_cast<uintptr_t>(x) & 15) == 0, len,
                lane, xn);
    }
    const float wi = w[i];
    double sq = 0.0;
#pragma unroll
    for (int k = 0; k < kFuseE; ++k) {
      const float d = __fsub_rn(xv[k], bv[k]);
      acc[k] = add_rn(acc[k], mul_rn(wi, d));
      sq = __fma_rn(double(d), double(d), sq);
    }
    sq = wave_sum(sq);
    if (lane == 0) partial[int64_t(c) * n + i] = sq;
  }
  }
#pragma unroll
  for (int k = 0; k < kFuseE; ++k) {
    const int idx = fuse_idx(lane, k);
    if (idx < len) out[start + idx] = acc[k];
  }
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

namespace {

int delta_wsum(const char *what, bool keys, const float *const *rows,
               const float *weights, int n, int64_t numel, const float *base,
               const float *const *base_keys, const int64_t *seg_off,
               int nseg, float *out, fsagg_stream_t stream) {
  if (!rows || !weights || !out || n < 1 || numel < 0 ||
      (keys ? (!base_keys || !seg_off || nseg < 1) : !base)) {
    set_error("%s: invalid argument (n=%d nseg=%d)", what, n, nseg);
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  const dim3 grid(unsigned((numel + 4 * kBlock - 1) / (4 * kBlock)));
  if (keys)
    hipLaunchKernelGGL(delta_wsum_kernel<true>, grid, dim3(kBlock), 0,
                       as_stream(stream), rows, weights, n, numel, nullptr,
                       base_keys, seg_off, nseg, out);
  else
    hipLaunchKernelGGL(delta_wsum_kernel<false>, grid, dim3(kBlock), 0,
                       as_stream(stream), rows, weights, n, numel, base,
                       nullptr, nullptr, 0, out);
  return check_launch(what);
}

int delta_sqnorm(const char *what, bool keys, const float *const *rows,
                 int n, int64_t numel, const float *base,
                 const float *const *base_keys, const int64_t *seg_off,
                 int nseg, double *sq, void *workspace,
                 size_t workspace_bytes, fsagg_stream_t stream) {
  if (!rows || !seg_off || !sq || n < 1 || nseg < 1 || numel < 0 ||
      delta_plan(numel, nseg).max_chunks > 65535) {
    set_error("%s: invalid argument (n=%d nseg=%d)", what, n, nseg);
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_delta_sqnorm_workspace_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu bytes", what, workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  const DeltaPlan pl = delta_plan(numel, nseg);
  int *prefix = static_cast<int *>(workspace);
  double *partial = reinterpret_cast<double *>(
      static_cast<char *>(workspace) + align256(sizeof(int) * size_t(nseg + 1)));
  hipLaunchKernelGGL(delta_prefix_kernel, dim3(1), dim3(1), 0, s, seg_off,
                     nseg, pl.chl, prefix);
  const dim3 grid(unsigned(n), unsigned(pl.max_chunks));
  if (keys)
    hipLaunchKernelGGL(delta_partial_kernel<true>, grid, dim3(kBlock), 0, s,
                       rows, nullptr, base_keys, seg_off, nseg, prefix,
                       pl.chl, partial, n);
  else
    hipLaunchKernelGGL(delta_partial_kernel<false>, grid, dim3(kBlock), 0, s,
                       rows, base, nullptr, seg_off, nseg, prefix, pl.chl,
                       partial, n);
  const int64_t waves = int64_t(n) * nseg;
  const int64_t per = kBlock / kWave;
  hipLaunchKernelGGL(delta_final_kernel, dim3(unsigned((waves + per - 1) / per)),
                     dim3(kBlock), 0, s, partial, prefix, nseg, n, sq);
  return check_launch(what);
}

}  // namespace

extern "C" int fsagg_delta_wsum_f32(const float *const *rows,
                                    const float *weights, int n,
                                    int64_t numel, const float *base,
                                    float *out, fsagg_stream_t stream) {
  return delta_wsum("fsagg_delta_wsum_f32", false, rows, weights, n, numel,
                    base, nullptr, nullptr, 0, out, stream);
}

extern "C" int fsagg_delta_wsum_keys_f32(const float *const *keys,
                                         const float *weights, int n,
                                         int64_t numel,
                                         const float *const *base_keys,
                                         const int64_t *seg_off, int nseg,
                                         float *out, fsagg_stream_t stream) {
  return delta_wsum("fsagg_delta_wsum_keys_f32", true, keys, weights, n,
                    numel, nullptr, base_keys, seg_off, nseg, out, stream);
}

extern "C" size_t fsagg_delta_sqnorm_workspace_bytes(int n, int64_t numel,
                                                     int nseg) {
  if (n < 1 || nseg < 1 || numel < 0) return 0;
  const DeltaPlan pl = delta_plan(numel, nseg);
  return align256(sizeof(int) * size_t(nseg + 1)) +
         align256(sizeof(double) * size_t(pl.max_chunks) * size_t(n));
}

extern "C" int fsagg_delta_sqnorm_f32(const float *const *rows, int n,
                                      int64_t numel, const float *base,
                                      const int64_t *seg_off, int nseg,
                                      double *sq, void *workspace,
                                      size_t workspace_bytes,
                                      fsagg_stream_t stream) {
  return delta_sqnorm("fsagg_delta_sqnorm_f32", false, rows, n, numel, base,
                      nullptr, seg_off, nseg, sq, workspace, workspace_bytes,
                      stream);
}

extern "C" int fsagg_delta_sqnorm_keys_f32(
    const float *const *keys, int n, int64_t numel,
    const float *const *base_keys, const int64_t *seg_off, int nseg,
    double *sq, void *workspace, size_t workspace_bytes,
    fsagg_stream_t stream) {
  return delta_sqnorm("fsagg_delta_sqnorm_keys_f32", true, keys, n, numel,
                      nullptr, base_keys, seg_off, nseg, sq, workspace,
                      workspace_bytes, stream);
}

namespace {

int64_t fused_max_chunks(int64_t numel, int nseg) {
  return numel / kFuseChunk + nseg + 1;
}

int delta_fused(const char *what, bool keys, const float *const *rows,
                const float *weights, int n, int64_t numel, const float *base,
                const float *const *base_keys, const int64_t *seg_off,
                int nseg, double *sq, float *out, void *workspace,
                size_t workspace_bytes, fsagg_stream_t stream) {
  if (!rows || !weights || !seg_off || !sq || !out || n < 1 || nseg < 1 ||
      numel < 0 || (keys ? !base_keys : !base) ||
      fused_max_chunks(numel, nseg) > (int64_t(1) << 30)) {
    set_error("%s: invalid argument (n=%d nseg=%d)", what, n, nseg);
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_delta_sqnorm_wsum_workspace_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu bytes", what, workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  const int64_t chunks = fused_max_chunks(numel, nseg);
  int *prefix = static_cast<int *>(workspace);
  double *partial = reinterpret_cast<double *>(
      static_cast<char *>(workspace) + align256(sizeof(int) * size_t(nseg + 1)));
  hipLaunchKernelGGL(delta_prefix_kernel, dim3(1), dim3(1), 0, s, seg_off,
                     nseg, int64_t(kFuseChunk), prefix);
  if (keys)
    hipLaunchKernelGGL(delta_fused_kernel<true>, dim3(unsigned(chunks)),
                       dim3(kWave), 0, s, rows, weights, n, nullptr,
                       base_keys, seg_off, nseg, prefix, partial, out);
  else
    hipLaunchKernelGGL(delta_fused_kernel<false>, dim3(unsigned(chunks)),
                       dim3(kWave), 0, s, rows, weights, n, base, nullptr,
                       seg_off, nseg, prefix, partial, out);
  const int64_t waves = int64_t(n) * nseg;
  const int64_t per = kBlock / kWave;
  hipLaunchKernelGGL(delta_final_kernel,
                     dim3(unsigned((waves + per - 1) / per)), dim3(kBlock), 0,
                     s, partial, prefix, nseg, n, sq);
  return check_launch(what);
}

}  // namespace

extern "C" size_t fsagg_delta_sqnorm_wsum_workspace_bytes(int n,
                                                          int64_t numel,
                                                          int nseg) {
  if (n < 1 || nseg < 1 || numel < 0) return 0;
  return align256(sizeof(int) * size_t(nseg + 1)) +
         align256(sizeof(double) * size_t(fused_max_chunks(numel, nseg)) *
                  size_t(n));
}

extern "C" int fsagg_delta_sqnorm_wsum_f32(
    const float *const *rows, const float *weights, int n, int64_t numel,
    const float *base, const int64_t *seg_off, int nseg, double *sq,
    float *out, void *workspace, size_t workspace_bytes,
    fsagg_stream_t stream) {
  return delta_fused("fsagg_delta_sqnorm_wsum_f32", false, rows, weights, n,
                     numel, base, nullptr, seg_off, nseg, sq, out, workspace,
                     workspace_bytes, stream);
}

extern "C" int fsagg_delta_sqnorm_wsum_keys_f32(
    const float *const *keys, const float *weights, int n, int64_t numel,
    const float *const *base_keys, const int64_t *seg_off, int nseg,
    double *sq, float *out, void *workspace, size_t workspace_bytes,
    fsagg_stream_t stream) {
  return delta_fused("fsagg_delta_sqnorm_wsum_keys_f32", true, keys, weights,
                     n, numel, nullptr, base_keys, seg_off, nseg, sq, out,
                     workspace, workspace_bytes, stream);
}
