// Krum distances of a few clients to every client, in fp64 (gfx950).
//
// The Gram path (pairgram.hip) gives every pair's distance with a bound on
// its error; when the bounds do not separate a Krum / Bulyan selection, only
// the clients whose score intervals straddle the cut are ambiguous
// (core/aggregators/_engine.refine_selection).  Their rows of the distance
// matrix — |sel| × n pairs, not n² — are recomputed here with fp64
// differences, squares and sums (relative error ~1e-10 at millions of
// coordinates), which makes those clients' Krum scores (krum_aggregator.py
// :58-77, a sum over the client's own row) points instead of intervals.
//
// Work decomposition
//   * the row set's chunk table (fsagg_chunk, FSAGG_PAIRSEL_CHUNK
//     coordinates, never straddling a key); one 256-thread workgroup per
//     chunk, walking it in stages of T coordinates (T = 8192 / the client
//     slots: 128 at n <= 64, 32 at n > 128).  2048-coordinate chunks: at
//     4096 the C4 grid (1612 workgroups, 4 per CU) ends in a 0.6-full
//     round — 2 rows of 50 clients × 6.6M took 0.279 against 0.251 ms
//     (1024: 0.267, 512: 0.324; tools/probe_pairsel.py);
//   * NA accumulator slots per lane, 2 / 4 / 8 / 16 / 32 (the one or two
//     rows of a typical near-tie take the 2-slot kernel: 0.279 against
//     0.348 ms on 4 slots);
//   * every client's stage is loaded coalesced (consecutive lanes read
//     consecutive 16-B pieces of one row) into registers one stage ahead,
//     then written to LDS transposed, [coordinate][client] at a pitch of
//     slots + 1 words (conflict-free reads; at most 2-way on the writes);
//     the selected rows' stage goes to LDS as fp64 [coordinate][a]
//     (pitch NA + 2 doubles), read as wave-uniform broadcasts (a readlane
//     per value instead — the selected rows lane-distributed in registers,
//     each value a scalar operand — measured 10-20 % slower at NA <= 8,
//     tools/probe_pairsel.py);
//   * lane ↔ client b (ceil(n/64) waves cover the clients, the other waves
//     take other coordinate slices of the stage); each lane keeps NA fp64
//     accumulators, one per selected client;
//   * after the chunk the coordinate slices are summed in slice order
//     through LDS → partial[chunk][a][b]; a wave per (key, a, b) adds the
//     key's chunks in a fixed order → segsq[key][a][b]; the finish kernel
//     takes Σ_key sqrt(segsq) in fp64 in key order.
// Deterministic: no atomics anywhere.
#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kMaxStage = 128;     // coordinates per stage (n <= 64)
constexpr int kRowFloats = 8320;   // the clients' stage: T × (slots + 1)

// client slots (whole waves) and stage length for n clients
__host__ __device__ inline int pairsel_slots(int n) {
  return (n + kWave - 1) / kWave * kWave;
}
__host__ __device__ inline int pairsel_stage(int n) {
  const int t = 8192 / pairsel_slots(n) / 16 * 16;
  return t > kMaxStage ? kMaxStage : t;
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

template <int NA>
__global__ __launch_bounds__(kBlock) void pairsel_chunk_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n,
    const int *__restrict__ sel, int nsel,
    const fsagg_chunk *__restrict__ chunks, double *__restrict__ partial) {
  constexpr int PA = NA + 2;  // doubles per staged coordinate of the rows a
  __shared__ __attribute__((aligned(16))) float lb[kRowFloats];
  __shared__ __attribute__((aligned(16))) double la[kMaxStage * PA];
  const int c = blockIdx.x;
  const int64_t lo = chunks[c].lo;
  const int len = chunks[c].len;
  const float *const *__restrict__ rows = tab + int64_t(chunks[c].seg) * ss;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid & (kWave - 1);
  const int slots = pairsel_slots(n), T = pairsel_stage(n);
  const int pb = slots + 1;  // LDS pitch (words) of a staged coordinate
  const int bset = slots / kWave;
  const int slices = kWaves / bset;
  const int slice = wave / bset;
  const int b = (wave - slice * bset) * kWave + lane;
  const bool busy = slice < slices;
  // row pointers at this chunk: the clients', then the selected rows'
  __shared__ const float *rp[FSAGG_PAIRSEL_MAX_CLIENTS + NA];
  for (int r = tid; r < n; r += kBlock) rp[r] = rows[r] + lo;
  for (int a = tid; a < NA; a += kBlock)
    rp[FSAGG_PAIRSEL_MAX_CLIENTS + a] = rows[sel[a < nsel ? a : nsel - 1]] + lo;
  // 16-B loads when every client row is aligned at this chunk (the barrier
  // also publishes rp)
  const bool vec = __syncthreads_and(
      tid >= n || (reinterpret_cast<uintptr_t>(rows[tid] + lo) & 15u) == 0);
  const float *const *sp = rp + FSAGG_PAIRSEL_MAX_CLIENTS;

  // Register staging of one whole stage.  The clients' rows as float4
  // units: thread tid takes piece q = tid % (T/4) of rows r0, r0 + rstep, …
  // (T/4 divides the block, so the piece is fixed); the selected rows as
  // floats: coordinate pa = tid % T of rows a0, a0 + astep, ….  At most 8
  // units (T·slots/4 <= 2048) and NA/2 floats per thread.
  constexpr int KB = 8;
  constexpr int KA = NA * kMaxStage / kBlock;
  const int q4 = T / 4;
  const int q = tid % q4, r0 = tid / q4, rstep = kBlock / q4;
  const int pa = tid % T, a0 = tid / T, astep = kBlock / T;
  f4v rb[KB];
  float ra[KA];
  auto fetch = [&](int s0) {
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int r = r0 + k * rstep;
      if (r < n) rb[k] = gld_nt(reinterpret_cast<const f4v *>(rp[r] + s0) + q);
    }
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int a = a0 + k * astep;
      if (a < NA) ra[k] = gld(sp[a] + s0 + pa);
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int r = r0 + k * rstep;
      if (r < n) {
        float *d = lb + 4 * q * pb + r;
        d[0] = rb[k].x;
        d[pb] = rb[k].y;
        d[2 * pb] = rb[k].z;
        d[3 * pb] = rb[k].w;
      }
    }
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int a = a0 + k * astep;
      if (a < NA) la[pa * PA + a] = double(ra[k]);
    }
  };
  // unaligned rows or a short tail stage: 4-B loads straight to LDS
  auto put_scalar = [&](int s0) {
    const int sl = len - s0 < T ? len - s0 : T;
    for (int u = tid; u < n * T; u += kBlock) {
      const int r = u / T, p = u - r * T;
      if (p < sl) lb[p * pb + r] = gld(rp[r] + s0 + p);
    }
    for (int i = tid; i < NA * T; i += kBlock) {
      const int a = i / T, p = i - a * T;
      if (p < sl) la[p * PA + a] = double(gld(sp[a] + s0 + p));
    }
  };
  auto whole = [&](int s0) { return vec && len - s0 >= T; };

  double acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.0;

  if (whole(0)) fetch(0);
  for (int s0 = 0; s0 < len; s0 += T) {
    if (whole(s0)) put();
    else put_scalar(s0);
    __syncthreads();
    if (whole(s0 + T)) fetch(s0 + T);  // lands while this stage computes
    if (busy) {
      const int sl = len - s0 < T ? len - s0 : T;
      const int per = T / slices;
      const int p0 = slice * per;
      const int p1 = p0 + per < sl ? p0 + per : sl;
#pragma unroll 2
      for (int p = p0; p < p1; ++p) {
        const double x = double(lb[p * pb + b]);
        const d2v *r = reinterpret_cast<const d2v *>(la + p * PA);
#pragma unroll
        for (int h = 0; h < NA / 2; ++h) {
          const d2v v = r[h];
          const double d0 = v.x - x, d1 = v.y - x;
          acc[2 * h] = __builtin_fma(d0, d0, acc[2 * h]);
          acc[2 * h + 1] = __builtin_fma(d1, d1, acc[2 * h + 1]);
        }
      }
    }
    __syncthreads();
  }

  // the slices' sums in slice order, 16 selected rows at a time (the
  // clients' stage region, as doubles: slices·16·slots = 4096 <= 4160)
  double *red = reinterpret_cast<double *>(lb);
  const int nb = slots;
  constexpr int G = NA < 16 ? NA : 16;
#pragma unroll
  for (int a0g = 0; a0g < NA; a0g += G) {
    if (busy) {
#pragma unroll
      for (int g = 0; g < G; ++g) red[(slice * G + g) * nb + b] = acc[a0g + g];
    }
    __syncthreads();
    for (int o = tid; o < G * nb; o += kBlock) {
      const int g = o / nb, bb = o - g * nb;
      const int a = a0g + g;
      if (bb >= n || a >= nsel) continue;
      double t = 0.0;
      for (int k = 0; k < slices; ++k) t += red[(k * G + g) * nb + bb];
      partial[(int64_t(c) * nsel + a) * n + bb] = t;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// One wave per (key, a, b): lane l adds the key's chunks first + l,
// first + l + 64, … in order, then a fixed shuffle tree.  The chunks of a
// key are contiguous in the table.
__global__ __launch_bounds__(kBlock) void pairsel_segsq_kernel(
    const fsagg_chunk *__restrict__ chunks, int nchunk, int n, int nsel,
    int nseg, const double *__restrict__ partial, double *__restrict__ segsq) {
  const int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t per_seg = int64_t(nsel) * n;
  if (q >= per_seg * nseg) return;  // whole waves leave together
  const int s = int(q / per_seg);
  const int64_t ab = q - s * per_seg;
  int lo = 0, hi = nchunk;  // first chunk with seg >= s
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (chunks[mid].seg < s) lo = mid + 1;
    else hi = mid;
  }
  int end = lo;  // first chunk with seg > s
  hi = nchunk;
  while (end < hi) {
    const int mid = (end + hi) >> 1;
    if (chunks[mid].seg <= s) end = mid + 1;
    else hi = mid;
  }
  double t = 0.0;
  for (int c = lo + lane; c < end; c += kWave) t += partial[c * per_seg + ab];
  t = wave_sum(t);
  if (lane == 0) segsq[q] = t;
}

// D[a][b] = Σ_key sqrt(segsq[key][a][b]) in fp64, key order; the selected
// client's own entry +inf (krum_aggregator.py:67-69).
__global__ __launch_bounds__(kBlock) void pairsel_finish_kernel(
    const double *__restrict__ segsq, const int *__restrict__ sel, int nsel,
    int n, int nseg, double *__restrict__ D) {
  const int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= nsel * n) return;
  const int a = q / n, b = q - a * n;
  if (b == sel[a]) {
    D[q] = __builtin_inf();
    return;
  }
  double t = 0.0;
  for (int s = 0; s < nseg; ++s)
    t += sqrt(segsq[int64_t(s) * nsel * n + q]);
  D[q] = t;
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" size_t fsagg_pairsel_workspace_bytes(int nsel, int n, int nchunk) {
  if (nsel < 1 || n < 1 || nchunk < 1) return 0;
  return sizeof(double) * size_t(nchunk) * size_t(nsel) * size_t(n);
}

extern "C" int fsagg_pairsel_rows_segsq_f64(const fsagg_rows *rows,
                                            const int *sel, int nsel,
                                            const fsagg_chunk *chunks,
                                            int nchunk, double *segsq,
                                            void *workspace,
                                            size_t workspace_bytes,
                                            fsagg_stream_t stream) {
  if (!rows || !rows->tab || rows->n < 2 ||
      rows->n > FSAGG_PAIRSEL_MAX_CLIENTS || rows->nseg < 1 || !sel ||
      nsel < 1 || nsel > FSAGG_PAIRSEL_MAX_SEL || !segsq || nchunk < 0 ||
      (nchunk > 0 && !chunks)) {
    set_error("fsagg_pairsel_rows_segsq_f64: invalid argument");
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_pairsel_workspace_bytes(nsel, rows->n, nchunk);
  if (need && (!workspace || workspace_bytes < need)) {
    set_error("fsagg_pairsel_rows_segsq_f64: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  double *partial = static_cast<double *>(workspace);
  if (nchunk > 0) {
#define FSAGG_PAIRSEL(NA)                                                     \
  hipLaunchKernelGGL(pairsel_chunk_kernel<NA>, dim3(unsigned(nchunk)),       \
                     dim3(kBlock), 0, s, rows->tab, rows->ss, rows->n, sel,  \
                     nsel, chunks, partial)
    if (nsel <= 2) FSAGG_PAIRSEL(2);
    else if (nsel <= 4) FSAGG_PAIRSEL(4);
    else if (nsel <= 8) FSAGG_PAIRSEL(8);
    else if (nsel <= 16) FSAGG_PAIRSEL(16);
    else FSAGG_PAIRSEL(32);
#undef FSAGG_PAIRSEL
  }
  const int64_t waves = int64_t(rows->nseg) * nsel * rows->n;
  const int64_t per = kBlock / kWave;
  hipLaunchKernelGGL(pairsel_segsq_kernel,
                     dim3(unsigned((waves + per - 1) / per)), dim3(kBlock), 0,
                     s, chunks, nchunk, rows->n, nsel, rows->nseg, partial,
                     segsq);
  return check_launch("fsagg_pairsel_rows_segsq_f64");
}

extern "C" int fsagg_pairsel_finish_f64(const double *segsq, const int *sel,
                                        int nsel, int n, int nseg, double *D,
                                        fsagg_stream_t stream) {
  if (!segsq || !sel || !D || nsel < 1 || n < 1 || nseg < 1) {
    set_error("fsagg_pairsel_finish_f64: invalid argument");
    return FSAGG_EINVAL;
  }
  hipLaunchKernelGGL(pairsel_finish_kernel,
                     dim3(unsigned((nsel * n + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, as_stream(stream), segsq, sel, nsel, n,
                     nseg, D);
  return check_launch("fsagg_pairsel_finish_f64");
}
