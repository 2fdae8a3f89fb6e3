// Krum pairwise distances on the matrix cores (gfx950 bf16 MFMA), n <= 64.
//
// Krum's distance between clients a and b is Σ_keys ‖x_a − x_b‖ over each
// key (krum_aggregator.py:41-56: `distance += torch.dist(a[key], b[key])`).
// The VALU kernel (pairdist.hip) forms every (x_a − x_b)² directly; it is
// issue-bound (floor 0.28 ms at C4).  Here the per-key squared
// distances come from a Gram matrix,
//     d²(a, b) = G_aa + G_bb − 2·G_ab,   G = Σ_p x'_a[p]·x'_b[p],
// computed on the matrix cores.  Two things keep it exact enough:
//
// * Every fp32 value is split into three bf16 limbs by truncation,
//   x = h + m + l exactly (8 + 8 + 8 significand bits); the six limb
//   products of weight ≥ 2^-16 (hh, hm, mh, hl, lh, mm) are exact in the
//   MFMA and the three dropped ones are < 2^-21 of |x_a·x_b|.  Each
//   k-step's six products of a tile pair are chained through the MFMA in
//   fp32 (small limbs first) and added into fp64 accumulators (a wave's
//   chunk); chunks are summed per key in fp64 in a fixed order.
// * The Gram form cancels (G_aa + G_bb ≫ d² for near-identical clients, the
//   very pairs Krum ranks), so the data are CENTRED on one client c first:
//   x' = x − x_c, exact by Sterbenz whenever x and x_c are within a factor
//   of two, which is when cancellation would matter.  c is the client with
//   the smallest sum of distances to the others over a sample of the
//   coordinates (the first kSampleCoords of every key) — a central client,
//   so (G'_aa + G'_bb) / d² stays O(1) for every pair near the centre.
//   Pairs whose predicted error is still too large (a cluster far from the
//   centre: near-duplicate or colluding clients) are flagged in ill[a][b];
//   the caller recomputes those pairs exactly on the VALU kernel.
//   Identical rows give d² = 0 exactly (identical sums).
//
// Work: one wave per chunk of <= W coordinates inside one key; its lanes
// load the 16-client tiles straight into MFMA fragment order (lane l:
// client 16t + (l&15), coordinates 8(l>>4) .. +7 of the k-step), so every
// value is read from HBM once and nothing goes through LDS.
#include "common.h"

namespace fsagg {
namespace {

typedef short frag8 __attribute__((ext_vector_type(8)));     // 8 bf16
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGramMaxTiles = 4;          // n <= 64
constexpr int kKStep = 32;                // coordinates per MFMA k-step
constexpr int kRed = 32;                  // chunks per first-level sum
constexpr int64_t kSampleCoords = 2048;   // per key, for the centre choice
constexpr int64_t kSampleChunk = 128;
// error model of d² = G'aa + G'bb − 2G'ab: relative error ≈ kErrCoef ·
// (G'aa + G'bb) / d² · sqrt(32 / key length) (fp32 roundings of the k-step
// sums, random in sign); pairs predicted above kErrTol are flagged
constexpr double kErrCoef = 1.8e-7;
constexpr double kErrTol = 2e-7;

constexpr int ntp_of(int nt) { return nt * (nt + 1) / 2; }

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

__device__ __forceinline__ bool al16(const float *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// chunks per key and their prefix: chunk q of key s covers
// [seg_lo[s] + q·w, min(seg_lo[s] + (q+1)·w, cap_s)), cap_s = seg_end[s]
// (or seg_lo[s] + kSampleCoords for the sample plan)
__global__ void gram_prefix_kernel(const int64_t *__restrict__ seg_lo,
                                   const int64_t *__restrict__ seg_end,
                                   int nseg, int64_t w, int64_t cap,
                                   int *prefix) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int acc = 0;
  prefix[0] = 0;
  for (int s = 0; s < nseg; ++s) {
    int64_t len = seg_end[s] - seg_lo[s];
    if (cap > 0 && len > cap) len = cap;
    if (len < 0) len = 0;
    // padded to whole groups of kRed chunks (empty chunks write zeros), so
    // a first-level sum never straddles two keys
    const int64_t c = (len + w - 1) / w;
    acc += int((c + kRed - 1) / kRed * kRed);
    prefix[s + 1] = acc;
  }
}

__device__ __forceinline__ void tp_tiles(int tp, int nt, int &t, int &u) {
  int r = 0, base = 0;
  while (tp >= base + (nt - r)) {
    base += nt - r;
    ++r;
  }
  t = r;
  u = r + (tp - base);
}

// Split 8 fp32 (already centred) into three packed bf16 limbs, each the
// round-to-nearest bf16 of what the previous limbs leave (x − h and
// x − h − m are exact in fp32): x = h + m + l to within 2^-24·|x|, with
// residuals of both signs (no bias in the dropped products).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_rne(float a, float b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_convertvector(f32x2{a, b}, bf16x2));
}

__device__ __forceinline__ void split3(const float (&x)[8], frag8 &h,
                                       frag8 &m, frag8 &l) {
  u32x4 ph, pm, pl;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t hp = pk_rne(a, b);
    const float ra = a - __uint_as_float(hp << 16);
    const float rb = b - __uint_as_float(hp & 0xffff0000u);
    const uint32_t mp = pk_rne(ra, rb);
    const float sa = ra - __uint_as_float(mp << 16);
    const float sb = rb - __uint_as_float(mp & 0xffff0000u);
    ph[p] = hp;
    pm[p] = mp;
    pl[p] = pk_rne(sa, sb);
  }
  h = __builtin_bit_cast(frag8, ph);
  m = __builtin_bit_cast(frag8, pm);
  l = __builtin_bit_cast(frag8, pl);
}

// Load 8 consecutive coordinates [k, k + 8) of `row` (a virtual base:
// bucket coordinate p is row[p]) clipped to [.., c1); zeros past c1 or for
// a missing row.  `vec`: both 16-B loads are aligned (checked per wave).
__device__ __forceinline__ void load8(const float *row, int64_t k, int64_t c1,
                                      bool vec, float (&v)[8]) {
  if (row == nullptr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.0f;
    return;
  }
  if (vec && k + 8 <= c1) {
    const f32x4 a = gld_nt(reinterpret_cast<const f32x4 *>(row + k));
    const f32x4 b = gld_nt(reinterpret_cast<const f32x4 *>(row + k + 4));
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = k + j < c1 ? gload(row + k + j) : 0.0f;
}

// One wave per chunk.  partial[chunk][tp][reg][lane] (fp64): the chunk's
// centred Gram blocks in MFMA C-layout (row 4(lane>>4) + reg of tile t,
// column lane&15 of tile u).  SAMPLE: centre = none (raw values).
template <int NT>
__global__ __launch_bounds__(kWave, 2) void gram_chunk_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, const int *__restrict__ prefix, int64_t w, int64_t cap,
    const int *__restrict__ centre, double *__restrict__ partial) {
  constexpr int NTP = ntp_of(NT);
  const int chunk = blockIdx.x;
  if (chunk >= prefix[nseg]) return;
  int s = 0;
  while (prefix[s + 1] <= chunk) ++s;
  const int q = chunk - prefix[s];
  const int lane = threadIdx.x;
  int64_t send = seg_end[s];
  if (cap > 0 && send > seg_lo[s] + cap) send = seg_lo[s] + cap;
  const int64_t c0 = seg_lo[s] + int64_t(q) * w;
  const int64_t c1 = min(c0 + w, send);
  const float *const *rows = tab + int64_t(s) * ss;
  const float *row[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = 16 * t + (lane & 15);
    row[t] = j < n ? rows[j] : nullptr;
  }
  const float *crow = centre ? rows[*centre] : nullptr;
  // 16-B loads when every lane's first address is aligned
  const int64_t kl = c0 + 8 * (lane >> 4);
  bool ok = true;
#pragma unroll
  for (int t = 0; t < NT; ++t)
    ok = ok && (row[t] == nullptr || al16(row[t] + kl));
  if (crow) ok = ok && al16(crow + kl);
  const bool vec = __all(ok);

  double acc64[NTP][4];
#pragma unroll
  for (int p = 0; p < NTP; ++p) {
#pragma unroll
    for (int r = 0; r < 4; ++r) acc64[p][r] = 0.0;
  }
  // two k-steps of loads in flight ahead of the one being multiplied
  float xn[NT][8], cn[8], xq[NT][8], cq[8];
  {
    const int64_t k = c0 + 8 * (lane >> 4);
    if (crow) load8(crow, k, c1, vec, cn);
#pragma unroll
    for (int t = 0; t < NT; ++t) load8(row[t], k, c1, vec, xn[t]);
    if (crow) load8(crow, k + kKStep, c1, vec, cq);
#pragma unroll
    for (int t = 0; t < NT; ++t) load8(row[t], k + kKStep, c1, vec, xq[t]);
  }
  for (int64_t k0 = c0; k0 < c1; k0 += kKStep) {
    // split this k-step (its raw values die here), rotate the pipeline and
    // issue the loads two k-steps ahead before the MFMAs
    frag8 fh[NT], fm[NT], fl[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (crow) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          xn[t][j] = row[t] ? xn[t][j] - cn[j] : 0.0f;
      }
      split3(xn[t], fh[t], fm[t], fl[t]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) cn[j] = cq[j];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) xn[t][j] = xq[t][j];
    if (k0 + 2 * kKStep < c1) {
      const int64_t k = k0 + 2 * kKStep + 8 * (lane >> 4);
      if (crow) load8(crow, k, c1, vec, cq);
#pragma unroll
      for (int t = 0; t < NT; ++t) load8(row[t], k, c1, vec, xq[t]);
    }
    // per tile pair: one k-step's six limb products in fp32 (the small
    // ones first, so their roundings happen at their own magnitude), then
    // into fp64 — one chain of 6 MFMAs, one accumulator live at a time
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
      int t, u;
      tp_tiles(p, NT, t, u);
      f32x4 c = {0.0f, 0.0f, 0.0f, 0.0f};
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[t], fm[u], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[t], fl[u], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fl[t], fh[u], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[t], fm[u], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fm[t], fh[u], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[t], fh[u], c, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc64[p][r] += double(c[r]);
    }
  }
  double *out = partial + int64_t(chunk) * NTP * 256;
#pragma unroll
  for (int p = 0; p < NTP; ++p) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      out[(p * 4 + r) * 64 + lane] = acc64[p][r];
  }
}

// Sum the chunk partials of each key in a fixed order, in two levels:
// level 1, grid (total / kRed, NTP): block b sums chunks [kRed·b, kRed·b +
// kRed) (one key, the plan pads keys to whole groups) into red[b][p][256];
// level 2, grid (nseg, NTP): each key's groups in order into
// G[seg][64][64] (both triangles).  all_in_one sums every group into one
// matrix (the sample plan).
template <int NT>
__global__ __launch_bounds__(256) void gram_reduce1_kernel(
    const double *__restrict__ partial, const int *__restrict__ prefix,
    int nseg, double *__restrict__ red) {
  constexpr int NTP = ntp_of(NT);
  const int b = blockIdx.x, p = blockIdx.y, e = threadIdx.x;
  if (b * kRed >= prefix[nseg]) return;
  double v[kRed];
#pragma unroll
  for (int q = 0; q < kRed; ++q)
    v[q] = partial[((int64_t(b) * kRed + q) * NTP + p) * 256 + e];
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < kRed; ++q) sum += v[q];
  red[(int64_t(b) * NTP + p) * 256 + e] = sum;
}

template <int NT>
__global__ __launch_bounds__(256) void gram_reduce2_kernel(
    const double *__restrict__ red, const int *__restrict__ prefix,
    int nseg, int all_in_one, double *__restrict__ G) {
  constexpr int NTP = ntp_of(NT);
  const int s = blockIdx.x, p = blockIdx.y;
  const int r = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b0 = (all_in_one ? 0 : prefix[s]) / kRed;
  const int b1 = (all_in_one ? prefix[nseg] : prefix[s + 1]) / kRed;
  double sum = 0.0;
  for (int b = b0; b < b1; ++b)
    sum += red[(int64_t(b) * NTP + p) * 256 + threadIdx.x];
  int t, u;
  tp_tiles(p, NT, t, u);
  const int a = 16 * t + 4 * (lane >> 4) + r;
  const int c = 16 * u + (lane & 15);
  double *gm = G + int64_t(s) * 64 * 64;
  gm[a * 64 + c] = sum;
  if (t != u) gm[c * 64 + a] = sum;
}

// The centre: argmin_a Σ_b sqrt(d²(a, b)) over the sample Gram (one block).
__global__ __launch_bounds__(64) void gram_centre_kernel(
    const double *__restrict__ G, int n, int *__restrict__ centre) {
  __shared__ double tot[64];
  const int a = threadIdx.x;
  double sum = 0.0;
  if (a < n) {
    for (int b = 0; b < n; ++b) {
      const double d2 = G[a * 64 + a] + G[b * 64 + b] - 2.0 * G[a * 64 + b];
      sum += d2 > 0.0 ? sqrt(d2) : 0.0;
    }
  }
  tot[a] = a < n ? sum : 1e308;
  __syncthreads();
  if (a == 0) {
    int best = 0;
    for (int b = 1; b < n; ++b)
      if (tot[b] < tot[best]) best = b;
    *centre = best;
  }
}

// segsq[s][a][b] = G_aa + G_bb − 2·G_ab (diag 0, clamped at 0).  ill[a][b]
// (n x n words) is set for a pair whose d² the error model puts above
// kErrTol in some key, or whose d² came out negative: the caller
// recomputes those pairs exactly.  An exact 0 (identical rows: identical
// sums) is exact.
__global__ __launch_bounds__(256) void gram_segsq_kernel(
    const double *__restrict__ G, const int64_t *__restrict__ seg_lo,
    const int64_t *__restrict__ seg_end, int n, int nseg,
    double *__restrict__ segsq, uint32_t *__restrict__ ill) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(nseg) * n * n) return;
  const int s = int(i / (int64_t(n) * n));
  const int a = int((i / n) % n), b = int(i % n);
  const double *g = G + int64_t(s) * 64 * 64;
  if (a == b) {
    segsq[i] = 0.0;
    return;
  }
  const double gaa = g[a * 64 + a], gbb = g[b * 64 + b];
  const double d2 = gaa + gbb - 2.0 * g[a * 64 + b];
  const double len = double(seg_end[s] - seg_lo[s]);
  if (len > 0.0) {
    const double err = kErrCoef * (gaa + gbb) * sqrt(32.0 / len);
    if (d2 < 0.0 || err > kErrTol * d2) ill[a * n + b] = 1u;
  }
  segsq[i] = d2 > 0.0 ? d2 : 0.0;
}

struct GramPlan {
  int nt;
  int64_t w;           // main chunk length
  int main_chunks;     // upper bound
  int sample_chunks;   // upper bound
};

GramPlan gram_plan(int n, int64_t numel, int nseg) {
  GramPlan pl;
  pl.nt = (n + 15) / 16;
  // ~4096 chunks: two rounds of waves at 2 waves per SIMD
  int64_t w = (numel + 4095) / 4096;
  w = (w + kKStep - 1) / kKStep * kKStep;
  if (w < 4 * kKStep) w = 4 * kKStep;
  pl.w = w;
  pl.main_chunks = int(numel / w) + nseg * kRed + 1;
  pl.sample_chunks = int(nseg * (((kSampleCoords + kSampleChunk - 1) /
                                  kSampleChunk + kRed - 1) / kRed * kRed));
  return pl;
}

struct GramWs {
  int *prefix_main, *prefix_sample, *centre;
  double *partial, *g_sample, *g_main, *red;
};

GramWs gram_ws(void *ws, int n, int64_t numel, int nseg) {
  const GramPlan pl = gram_plan(n, numel, nseg);
  const int ntp = ntp_of(pl.nt);
  char *p = static_cast<char *>(ws);
  GramWs w;
  w.prefix_main = reinterpret_cast<int *>(p);
  p += align256(sizeof(int) * size_t(nseg + 1));
  w.prefix_sample = reinterpret_cast<int *>(p);
  p += align256(sizeof(int) * size_t(nseg + 1));
  w.centre = reinterpret_cast<int *>(p);
  p += 256;
  w.g_sample = reinterpret_cast<double *>(p);
  p += align256(sizeof(double) * 64 * 64);
  w.g_main = reinterpret_cast<double *>(p);
  p += align256(sizeof(double) * 64 * 64 * size_t(nseg));
  w.red = reinterpret_cast<double *>(p);
  p += align256(sizeof(double) * size_t(pl.main_chunks / kRed + 1) *
                size_t(ntp) * 256);
  w.partial = reinterpret_cast<double *>(p);
  return w;
}

size_t gram_ws_bytes(int n, int64_t numel, int nseg) {
  const GramPlan pl = gram_plan(n, numel, nseg);
  const size_t ntp = size_t(ntp_of(pl.nt));
  const size_t chunks = size_t(pl.main_chunks > pl.sample_chunks
                                   ? pl.main_chunks
                                   : pl.sample_chunks);
  return 2 * align256(sizeof(int) * size_t(nseg + 1)) + 256 +
         align256(sizeof(double) * 64 * 64) +
         align256(sizeof(double) * 64 * 64 * size_t(nseg)) +
         align256(sizeof(double) * size_t(pl.main_chunks / kRed + 1) * ntp *
                  256) +
         align256(sizeof(double) * chunks * ntp * 256);
}

template <int NT>
void gram_launch(const float *const *tab, int64_t ss, int n,
                 const int64_t *seg_lo, const int64_t *seg_end, int nseg,
                 const GramPlan &pl, const GramWs &w, double *segsq,
                 uint32_t *ill, hipStream_t st) {
  constexpr int NTP = ntp_of(NT);
  // 1. the centre: Gram of the first kSampleCoords of every key, raw
  hipLaunchKernelGGL(gram_prefix_kernel, dim3(1), dim3(1), 0, st, seg_lo,
                     seg_end, nseg, kSampleChunk, kSampleCoords,
                     w.prefix_sample);
  hipLaunchKernelGGL((gram_chunk_kernel<NT>), dim3(unsigned(pl.sample_chunks)),
                     dim3(kWave), 0, st, tab, ss, n, seg_lo, seg_end, nseg,
                     w.prefix_sample, kSampleChunk, kSampleCoords,
                     static_cast<const int *>(nullptr), w.partial);
  (void)hipMemsetAsync(w.g_sample, 0, sizeof(double) * 64 * 64, st);
  hipLaunchKernelGGL((gram_reduce1_kernel<NT>),
                     dim3(unsigned(pl.sample_chunks / kRed), unsigned(NTP)),
                     dim3(256), 0, st, w.partial, w.prefix_sample, nseg,
                     w.red);
  hipLaunchKernelGGL((gram_reduce2_kernel<NT>), dim3(1, unsigned(NTP)),
                     dim3(256), 0, st, w.red, w.prefix_sample, nseg, 1,
                     w.g_sample);
  hipLaunchKernelGGL(gram_centre_kernel, dim3(1), dim3(64), 0, st, w.g_sample,
                     n, w.centre);
  // 2. the centred Gram of every key
  hipLaunchKernelGGL(gram_prefix_kernel, dim3(1), dim3(1), 0, st, seg_lo,
                     seg_end, nseg, pl.w, int64_t(0), w.prefix_main);
  hipLaunchKernelGGL((gram_chunk_kernel<NT>), dim3(unsigned(pl.main_chunks)),
                     dim3(kWave), 0, st, tab, ss, n, seg_lo, seg_end, nseg,
                     w.prefix_main, pl.w, int64_t(0),
                     static_cast<const int *>(w.centre), w.partial);
  (void)hipMemsetAsync(w.g_main, 0, sizeof(double) * 64 * 64 * size_t(nseg),
                      st);
  hipLaunchKernelGGL((gram_reduce1_kernel<NT>),
                     dim3(unsigned(pl.main_chunks / kRed + 1), unsigned(NTP)),
                     dim3(256), 0, st, w.partial, w.prefix_main, nseg, w.red);
  hipLaunchKernelGGL((gram_reduce2_kernel<NT>),
                     dim3(unsigned(nseg), unsigned(NTP)), dim3(256), 0, st,
                     w.red, w.prefix_main, nseg, 0, w.g_main);
  const int64_t tot = int64_t(nseg) * n * n;
  hipLaunchKernelGGL(gram_segsq_kernel, dim3(unsigned((tot + 255) / 256)),
                     dim3(256), 0, st, w.g_main, seg_lo, seg_end, n, nseg,
                     segsq, ill);
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" size_t fsagg_pairgram_workspace_bytes(int n, int64_t numel,
                                                 int nseg) {
  if (n < 2 || n > 16 * kGramMaxTiles || nseg < 1 || numel < 0) return 0;
  return gram_ws_bytes(n, numel, nseg);
}

extern "C" int fsagg_pairgram_rows_segsq_f32(const fsagg_rows *rows,
                                             const int64_t *seg_lo,
                                             const int64_t *seg_end,
                                             int64_t numel, double *segsq,
                                             uint32_t *ill, void *workspace,
                                             size_t workspace_bytes,
                                             fsagg_stream_t stream) {
  if (!rows || !rows->tab || !seg_lo || !seg_end || !segsq || !ill ||
      rows->n < 2 || rows->n > 16 * kGramMaxTiles || rows->nseg < 1 ||
      numel < 0 || (rows->ss != 0 && rows->ss < rows->n)) {
    set_error("fsagg_pairgram_rows_segsq_f32: invalid argument (n must be "
              "2..%d)", 16 * kGramMaxTiles);
    return FSAGG_EINVAL;
  }
  const int n = rows->n, nseg = rows->nseg;
  const size_t need = gram_ws_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_pairgram_rows_segsq_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  const GramPlan pl = gram_plan(n, numel, nseg);
  const GramWs w = gram_ws(workspace, n, numel, nseg);
  hipStream_t st = as_stream(stream);
  switch (pl.nt) {
    case 1: gram_launch<1>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, ill, st); break;
    case 2: gram_launch<2>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, ill, st); break;
    case 3: gram_launch<3>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, ill, st); break;
    default: gram_launch<4>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                            w, segsq, ill, st); break;
  }
  return check_launch("fsagg_pairgram_rows_segsq_f32");
}
