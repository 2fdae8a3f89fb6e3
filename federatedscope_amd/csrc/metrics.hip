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

__global__ __launch_bounds__(kBlock) void delta_partial_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ base,
    const int64_t *__restrict__ seg_off, int nseg,
    const int *__restrict__ prefix, int64_t chl, double *__restrict__ partial,
    int n) {
  __shared__ double red[kBlock / kWave];
  const int c = blockIdx.x, row = blockIdx.y;
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
  const float *x = rows[row];
  double acc = 0.0;
  for (int64_t p = start + threadIdx.x; p < end; p += kBlock) {
    const float g = base ? __fsub_rn(x[p], base[p]) : x[p];
    acc += double(g) * double(g);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) t += red[w];
    partial[int64_t(c) * n + row] = t;
  }
}

// sq[row][s] = Σ over segment s's chunks (chunk order)
__global__ void delta_final_kernel(const double *__restrict__ partial,
                                   const int *__restrict__ prefix, int nseg,
                                   int n, double *__restrict__ sq) {
  const int64_t q = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= int64_t(n) * nseg) return;
  const int row = int(q / nseg), s = int(q % nseg);
  double t = 0.0;
  for (int c = prefix[s]; c < prefix[s + 1]; ++c)
    t += partial[int64_t(c) * n + row];
  sq[q] = t;
}

// out[p] = Σ_i fl32(w_i * fl32(x_i[p] - base[p])), list order, from +0:
// the global update of calc_blocal_dissim (metric_calculator.py:342-349).
__global__ __launch_bounds__(kBlock) void delta_wsum_kernel(
    const float *const *__restrict__ rows, const float *__restrict__ w, int n,
    int64_t numel, const float *__restrict__ base, float *__restrict__ out) {
  const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= numel) return;
  const float b = base[p];
  float acc = 0.0f;
  for (int i = 0; i < n; ++i)
    acc = add_rn(acc, mul_rn(w[i], __fsub_rn(rows[i][p], b)));
  out[p] = acc;
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_delta_wsum_f32(const float *const *rows,
                                    const float *weights, int n,
                                    int64_t numel, const float *base,
                                    float *out, fsagg_stream_t stream) {
  if (!rows || !weights || !base || !out || n < 1 || numel < 0) {
    set_error("fsagg_delta_wsum_f32: invalid argument (n=%d)", n);
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  hipLaunchKernelGGL(delta_wsum_kernel,
                     dim3(unsigned((numel + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, as_stream(stream), rows, weights, n,
                     numel, base, out);
  return check_launch("fsagg_delta_wsum_f32");
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
  if (!rows || !seg_off || !sq || n < 1 || nseg < 1 || numel < 0 ||
      n > 65535) {
    set_error("fsagg_delta_sqnorm_f32: invalid argument (n=%d nseg=%d)", n,
              nseg);
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_delta_sqnorm_workspace_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_delta_sqnorm_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  const DeltaPlan pl = delta_plan(numel, nseg);
  int *prefix = static_cast<int *>(workspace);
  double *partial = reinterpret_cast<double *>(
      static_cast<char *>(workspace) + align256(sizeof(int) * size_t(nseg + 1)));
  hipLaunchKernelGGL(delta_prefix_kernel, dim3(1), dim3(1), 0, s, seg_off,
                     nseg, pl.chl, prefix);
  hipLaunchKernelGGL(delta_partial_kernel,
                     dim3(unsigned(pl.max_chunks), unsigned(n)), dim3(kBlock),
                     0, s, rows, base, seg_off, nseg, prefix, pl.chl, partial,
                     n);
  const int64_t items = int64_t(n) * nseg;
  hipLaunchKernelGGL(delta_final_kernel,
                     dim3(unsigned((items + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, s, partial, prefix, nseg, n, sq);
  return check_launch("fsagg_delta_sqnorm_f32");
}
