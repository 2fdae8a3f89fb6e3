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
// * Every fp32 value is split exactly into three bf16 limbs, x = h + m + l
//   (each the round-to-nearest bf16 of what the previous ones leave; the
//   residuals x − h and x − h − m are exact in fp32 and come from one
//   v_dot2c_f32_bf16 each).  The six limb products of weight >= 2^-16 (hh,
//   hm, mh, hl, lh, mm) are exact in the MFMA; the dropped ones are
//   < 2^-24 of |x_a·x_b|.  Each k-step's six products of a tile pair are
//   chained through the MFMA in fp32 (small limbs first) and added into fp64
//   accumulators; the four waves of a workgroup are summed in LDS and the
//   chunks of a key in fp64 in a fixed order (deterministic).
// * The Gram form cancels (G_aa + G_bb ≫ d² for near-identical clients, the
//   very pairs Krum ranks), so the data are CENTRED on one client c first:
//   x' = x − x_c, exact by Sterbenz whenever x and x_c are within a factor
//   of two, which is when cancellation would matter.  c is the client with
//   the smallest sum of distances to the others over a sample of the
//   coordinates (the first kSampleCoords of every key) — a central client,
//   so (G'_aa + G'_bb) / d² stays O(1) for every pair near the centre.
//   Every per-key d² leaves with a predicted error bound err (the fp32
//   roundings of the k-step sums), and fsagg_pairgram_finish_f32 flags the
//   pairs whose Krum distance (the sum over keys) that bound could move by
//   more than the tolerance — a cluster far from the centre (near-duplicate
//   or colluding clients), or a non-finite value; the caller recomputes
//   those pairs exactly on the VALU kernel.
//
// Work: a workgroup of 4 waves per chunk of one key; wave v takes the
// chunk's k-steps v, v + 4, ...  A lane loads its 16-client tile rows
// straight into MFMA fragment order (lane l: client 16t + (l & 15); fragment
// slots 0-3 = coordinates 4(l>>4) .. +3 and slots 4-7 = 16 + 4(l>>4) .. +3
// of the k-step — any permutation of k is a valid contraction as long as
// both operands use it), so each load instruction reads 64 contiguous bytes
// of 16 rows, every value is read from HBM once and nothing goes through
// LDS on the way in.
#include "common.h"

namespace fsagg {
namespace {

typedef short frag8 __attribute__((ext_vector_type(8)));     // 8 bf16
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kGramMaxTiles = 4;          // n <= 64
constexpr int kKStep = 32;                // coordinates per MFMA k-step
constexpr int kWaves = 4;                 // waves per workgroup (chunk)
constexpr int kBlk = kWaves * kWave;
constexpr int64_t kUnit = kKStep * kWaves;  // chunk lengths: multiples
constexpr int kRed = 32;                  // chunks per first-level sum
constexpr int kMainChunks = 1024;         // ~2 rounds at 2 blocks per CU
constexpr int64_t kMaxW = 16384;          // chunk length cap (LDS centre)
constexpr int64_t kSampleCoords = 2048;   // per key, for the centre choice
constexpr int64_t kSampleChunk = 512;
// error model of d² = G'aa + G'bb − 2G'ab over a key of K k-steps: a part
// random in sign, kErrCoef · (G'aa + G'bb) / sqrt(K) (the fp32 roundings of
// the k-step sums; measured up to 2.4e-7 · (G'aa + G'bb) / sqrt(K) at C4),
// which err carries, and a part proportional to d² itself that the finish
// adds (fsagg_pairgram_finish_f32: 2e-8 · d², measured up to 3.6e-9 · d²;
// DESIGN §3.3)
constexpr double kErrCoef = 5e-7;
constexpr double kErrBias = 2e-8;

constexpr int ntp_of(int nt) { return nt * (nt + 1) / 2; }

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Chunks and first-level groups per key: chunk q of key s covers
// [seg_lo[s] + q·w, min(seg_lo[s] + (q+1)·w, cap_s)), cap_s = seg_end[s]
// (or seg_lo[s] + cap for the sample plan).  Group b of key s sums its
// chunks kRed·b .. kRed·b + kRed − 1.
__global__ void gram_prefix_kernel(const int64_t *__restrict__ seg_lo,
                                   const int64_t *__restrict__ seg_end,
                                   int nseg, int64_t w, int64_t cap,
                                   int *prefix, int *gprefix) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int acc = 0, gacc = 0;
  prefix[0] = 0;
  gprefix[0] = 0;
  for (int s = 0; s < nseg; ++s) {
    int64_t len = seg_end[s] - seg_lo[s];
    if (cap > 0 && len > cap) len = cap;
    if (len < 0) len = 0;
    const int c = int((len + w - 1) / w);
    acc += c;
    gacc += (c + kRed - 1) / kRed;
    prefix[s + 1] = acc;
    gprefix[s + 1] = gacc;
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

__device__ __forceinline__ uint32_t pk_rne(float a, float b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_convertvector(f32x2{a, b}, bf16x2));
}

// a − (low bf16 of hp), b − (high bf16 of hp): exact (each bf16 is the
// rounding of the fp32 it is taken from), one dot2 each.  nlo / nhi hold
// the bf16 pairs (−1, 0) and (0, −1) in VGPRs (Neg): as a literal the
// compiler folds (−1, 0) into the inline constant −1.0, which the hardware
// reads as fp32 bits 0xbf800000, i.e. (0, −1).
struct Neg {
  uint32_t lo, hi;
};
__device__ __forceinline__ Neg neg_consts() {
  Neg k{0x0000bf80u, 0xbf800000u};
  asm volatile("" : "+v"(k.lo), "+v"(k.hi));
  return k;
}
__device__ __forceinline__ float res_lo(uint32_t hp, float a, const Neg &k) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hp),
                                         __builtin_bit_cast(bf16x2, k.lo), a,
                                         false);
}
__device__ __forceinline__ float res_hi(uint32_t hp, float b, const Neg &k) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, hp),
                                         __builtin_bit_cast(bf16x2, k.hi), b,
                                         false);
}

// Split 8 fp32 into three packed bf16 limbs: x = h + m + l to within
// 2^-24·|x|, residuals of both signs (no bias in the dropped products).
__device__ __forceinline__ void split3(const float (&x)[8], const Neg &k,
                                       frag8 &h, frag8 &m, frag8 &l) {
  u32x4 ph, pm, pl;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t hp = pk_rne(a, b);
    const float ra = res_lo(hp, a, k), rb = res_hi(hp, b, k);
    const uint32_t mp = pk_rne(ra, rb);
    const float sa = res_lo(mp, ra, k), sb = res_hi(mp, rb, k);
    ph[p] = hp;
    pm[p] = mp;
    pl[p] = pk_rne(sa, sb);
  }
  h = __builtin_bit_cast(frag8, ph);
  m = __builtin_bit_cast(frag8, pm);
  l = __builtin_bit_cast(frag8, pl);
}

// fragment slot j of lane group g holds coordinate kofs(g, j) of a k-step
__device__ __forceinline__ bool al16(const float *p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

__device__ __forceinline__ int kofs(int g, int j) {
  return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
}

// One k-step in two phases.  kstep_split: centre (CENTRED: cs = the LDS
// centre values at this lane's coordinates of the k-step, slots 0-3 at cs,
// 4-7 at cs + 16) and split into limbs; kstep_mfma: the tile pairs'
// products into acc.
template <int NT>
struct Frags {
  frag8 h[NT], m[NT], l[NT];
};

template <int NT, bool CENTRED>
__device__ __forceinline__ void kstep_split(const float (&xb)[NT][8],
                                            const float *cs, const Neg &k,
                                            Frags<NT> &f) {
  float cb[8];
  if (CENTRED) {
    const f32x4 x = *reinterpret_cast<const f32x4 *>(cs);
    const f32x4 y = *reinterpret_cast<const f32x4 *>(cs + 16);
    cb[0] = x.x; cb[1] = x.y; cb[2] = x.z; cb[3] = x.w;
    cb[4] = y.x; cb[5] = y.y; cb[6] = y.z; cb[7] = y.w;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = CENTRED ? xb[t][j] - cb[j] : xb[t][j];
    split3(x, k, f.h[t], f.m[t], f.l[t]);
  }
}

// per tile pair: the six limb products in fp32 (the small ones first, so
// their roundings happen at their own magnitude), then into fp64
template <int NT>
__device__ __forceinline__ void kstep_mfma(const Frags<NT> &f,
                                           double (&acc)[ntp_of(NT)][4]) {
#pragma unroll
  for (int p = 0; p < ntp_of(NT); ++p) {
    int t, u;
    tp_tiles(p, NT, t, u);
    f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.m[t], f.m[u], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[t], f.l[u], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l[t], f.h[u], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[t], f.m[u], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.m[t], f.h[u], x, 0, 0, 0);
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[t], f.h[u], x, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[p][r] += double(x[r]);
  }
}

template <int NT, bool CENTRED>
__device__ __forceinline__ void kstep(const float (&xb)[NT][8],
                                      const float *cs, const Neg &k,
                                      double (&acc)[ntp_of(NT)][4]) {
  Frags<NT> f;
  kstep_split<NT, CENTRED>(xb, cs, k, f);
  kstep_mfma<NT>(f, acc);
}

// 16-B loads of one full k-step: slots 0-3 at a, 4-7 at a + 16
__device__ __forceinline__ void ld8(const float *a, float (&v)[8]) {
  const f32x4 x = gld_nt(reinterpret_cast<const f32x4 *>(a));
  const f32x4 y = gld_nt(reinterpret_cast<const f32x4 *>(a + 16));
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

// element loads of the k-step at k0 clipped to c1 (zeros past it)
__device__ __forceinline__ void ld8_tail(const float *row, int64_t k0,
                                         int64_t c1, int g, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t k = k0 + kofs(g, j);
    v[j] = k < c1 ? gload(row + k) : 0.0f;
  }
}

// One workgroup (4 waves) per chunk.  partial[chunk][tp][reg][lane] (fp64):
// the chunk's (centred) Gram blocks in MFMA C-layout (row 4(lane>>4) + reg
// of tile t, column lane & 15 of tile u).  !CENTRED: raw values (sample).
// The centre's values of the chunk (<= kMaxW) are staged in LDS once and
// read by every wave (registers go to the k-steps in flight).
template <int NT, bool CENTRED>
__global__ __launch_bounds__(kBlk, 2) void gram_chunk_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, const int *__restrict__ prefix, int64_t w, int64_t cap,
    const int *__restrict__ centre, double *__restrict__ partial) {
  constexpr int NTP = ntp_of(NT);
  constexpr int kRedWords = 2 * NTP * 4 * kWave;   // two waves' sums
  constexpr int kSmem = kRedWords * 8 > kMaxW * 4 ? kRedWords * 8
                                                   : int(kMaxW) * 4;
  __shared__ __attribute__((aligned(16))) char smem[kSmem];
  double(*red)[NTP * 4][kWave] =
      reinterpret_cast<double(*)[NTP * 4][kWave]>(smem);
  float *cs = reinterpret_cast<float *>(smem);
  const int chunk = blockIdx.x;
  if (chunk >= prefix[nseg]) return;   // whole workgroup
  int s = 0;
  while (prefix[s + 1] <= chunk) ++s;
  const int q = chunk - prefix[s];
  const int wv = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int g = lane >> 4;
  int64_t send = seg_end[s];
  if (cap > 0 && send > seg_lo[s] + cap) send = seg_lo[s] + cap;
  const int64_t c0 = seg_lo[s] + int64_t(q) * w;
  const int64_t c1 = min(c0 + w, send);
  const float *const *rows = tab + int64_t(s) * ss;
  // rows past n repeat row n − 1 (in the same tile, so the same load
  // instruction fetches it: no extra traffic); their Gram entries are
  // never read
  const float *row[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = 16 * t + (lane & 15);
    row[t] = rows[j < n ? j : n - 1];
  }

  double acc[NTP][4];
#pragma unroll
  for (int p = 0; p < NTP; ++p) {
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[p][r] = 0.0;
  }

  const Neg kn = neg_consts();
  const int64_t len = c1 > c0 ? c1 - c0 : 0;
  const int nfull = int(len / kKStep);
  // 16-B loads when every row's first address is aligned (per wave: the
  // waves' offsets differ by whole k-steps)
  bool ok = true;
#pragma unroll
  for (int t = 0; t < NT; ++t) ok = ok && al16(row[t] + c0);
  const bool vec = __all(ok);
  int i = wv;   // this wave's next k-step: wv, wv + 4, ...
  // one buffer: the next k-step's loads go out as soon as this one is split
  // and fly while its products are formed (the load depth of a ping-pong
  // pair of buffers measured the same); the first is issued
  // before the centre staging
  constexpr int64_t stp = int64_t(kWaves) * kKStep;
  const float *a[NT];
  float xa[NT][8];
  if (vec) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
      a[t] = row[t] + c0 + int64_t(i) * kKStep + 4 * g;
    if (i < nfull) {
#pragma unroll
      for (int t = 0; t < NT; ++t) ld8(a[t], xa[t]);
    }
  }
  if (CENTRED) {
    const float *crow = rows[*centre] + c0;
    if (al16(crow)) {
      for (int e = 4 * int(threadIdx.x); e < len; e += 4 * kBlk) {
        if (e + 4 <= len) {
          *reinterpret_cast<f32x4 *>(cs + e) =
              gld(reinterpret_cast<const f32x4 *>(crow + e));
        } else {
          for (int j = e; j < len; ++j) cs[j] = gload(crow + j);
        }
      }
    } else {
      for (int e = int(threadIdx.x); e < len; e += kBlk) cs[e] = gload(crow + e);
    }
    __syncthreads();
  }
  if (vec) {
    for (; i < nfull; i += kWaves) {
      Frags<NT> f;
      kstep_split<NT, CENTRED>(xa, cs + i * kKStep + 4 * g, kn, f);
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (the last k-step re-reads itself, from L2): a load
      // under a branch would make the buffer a phi and cost a copy of it
      const int64_t adv = i + kWaves < nfull ? stp : 0;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        a[t] += adv;
        ld8(a[t], xa[t]);
      }
      __builtin_amdgcn_sched_barrier(0);
      kstep_mfma<NT>(f, acc);
    }
    i = nfull + ((wv - nfull) % kWaves + kWaves) % kWaves;
  }
  // unaligned rows: every k-step; aligned: the partial last one (if any)
  const int nall = int((len + kKStep - 1) / kKStep);
  for (; i < nall; i += kWaves) {
    const int64_t k0 = c0 + int64_t(i) * kKStep;
    float xt[NT][8];
    __attribute__((aligned(16))) float ct[32];
#pragma unroll
    for (int t = 0; t < NT; ++t) ld8_tail(row[t], k0, c1, g, xt[t]);
    if (CENTRED) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int o = kofs(g, j);
        ct[o] = i * kKStep + o < len ? cs[i * kKStep + o] : 0.0f;
      }
    }
    kstep<NT, CENTRED>(xt, ct + 4 * g, kn, acc);
  }
  // the four waves' sums in a fixed order, (w0 + w2) + (w1 + w3), through
  // two wave-slots of LDS (red overlays the centre)
  if (CENTRED) __syncthreads();
  if (wv >= 2) {
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wv - 2][p * 4 + r][lane] = acc[p][r];
    }
  }
  __syncthreads();
  if (wv < 2) {
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[p][r] += red[wv][p * 4 + r][lane];
    }
  }
  __syncthreads();
  if (wv == 1) {
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[0][p * 4 + r][lane] = acc[p][r];
    }
  }
  __syncthreads();
  if (wv == 0) {
    double *out = partial + int64_t(chunk) * NTP * 256;
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(p * 4 + r) * 64 + lane] = acc[p][r] + red[0][p * 4 + r][lane];
    }
  }
}

// Level 1, grid (groups, NTP): group b (of key s) sums its <= kRed chunks
// in order into red[b][p][256].
template <int NT>
__global__ __launch_bounds__(256) void gram_reduce1_kernel(
    const double *__restrict__ partial, const int *__restrict__ prefix,
    const int *__restrict__ gprefix, int nseg, double *__restrict__ red) {
  constexpr int NTP = ntp_of(NT);
  const int b = blockIdx.x, p = blockIdx.y, e = threadIdx.x;
  if (b >= gprefix[nseg]) return;
  int s = 0;
  while (gprefix[s + 1] <= b) ++s;
  const int q0 = prefix[s] + (b - gprefix[s]) * kRed;
  const int q1 = min(q0 + kRed, prefix[s + 1]);
  double v[kRed];
#pragma unroll
  for (int q = 0; q < kRed; ++q)
    v[q] = q0 + q < q1 ? partial[((int64_t(q0) + q) * NTP + p) * 256 + e]
                       : 0.0;
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < kRed; ++q) sum += v[q];
  red[(int64_t(b) * NTP + p) * 256 + e] = sum;
}

// Level 2, grid (nseg or 1, NTP): each key's groups in order into
// G[seg][64][64] (both triangles of the tile pairs); all_in_one sums every
// group into one matrix (the sample plan).
template <int NT>
__global__ __launch_bounds__(256) void gram_reduce2_kernel(
    const double *__restrict__ red, const int *__restrict__ gprefix,
    int nseg, int all_in_one, double *__restrict__ G) {
  constexpr int NTP = ntp_of(NT);
  constexpr int U = 8;
  const int s = blockIdx.x, p = blockIdx.y;
  const int r = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b0 = all_in_one ? 0 : gprefix[s];
  const int b1 = all_in_one ? gprefix[nseg] : gprefix[s + 1];
  double sum = 0.0;
  for (int b = b0; b < b1; b += U) {
    double v[U];
#pragma unroll
    for (int j = 0; j < U; ++j)
      v[j] = b + j < b1 ? red[(int64_t(b + j) * NTP + p) * 256 + threadIdx.x]
                        : 0.0;
#pragma unroll
    for (int j = 0; j < U; ++j) sum += v[j];
  }
  int t, u;
  tp_tiles(p, NT, t, u);
  const int a = 16 * t + 4 * (lane >> 4) + r;
  const int c = 16 * u + (lane & 15);
  double *gm = G + int64_t(s) * 64 * 64;
  gm[a * 64 + c] = sum;
  if (t != u) gm[c * 64 + a] = sum;
}

// The centre: argmin_a Σ_b sqrt(d²(a, b)) over the sample Gram.
__global__ __launch_bounds__(256) void gram_centre_kernel(
    const double *__restrict__ G, int n, int *__restrict__ centre) {
  __shared__ double part[4][64];
  const int a = threadIdx.x & 63, h = threadIdx.x >> 6;
  double sum = 0.0;
  if (a < n) {
    const double gaa = G[a * 64 + a];
    for (int b = h; b < n; b += 4) {
      const double d2 = gaa + G[b * 64 + b] - 2.0 * G[a * 64 + b];
      sum += d2 > 0.0 ? sqrt(d2) : 0.0;
    }
  }
  part[h][a] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int best = 0;
    double bv = 0.0;
    for (int b = 0; b < n; ++b) {
      const double v = ((part[0][b] + part[1][b]) + part[2][b]) + part[3][b];
      if (b == 0 || v < bv) {
        bv = v;
        best = b;
      }
    }
    *centre = best;
  }
}

// segsq[s][a][b] = G_aa + G_bb − 2·G_ab (diag 0, clamped at 0) and its
// predicted absolute error err[s][a][b] (+inf when d² came out negative
// beyond that bound or is not finite: the pair is recomputed).
__global__ __launch_bounds__(256) void gram_segsq_kernel(
    const double *__restrict__ G, const int64_t *__restrict__ seg_lo,
    const int64_t *__restrict__ seg_end, int n, int nseg,
    double *__restrict__ segsq, double *__restrict__ err) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= int64_t(nseg) * n * n) return;
  const int s = int(i / (int64_t(n) * n));
  const int a = int((i / n) % n), b = int(i % n);
  const double *g = G + int64_t(s) * 64 * 64;
  if (a == b) {
    segsq[i] = 0.0;
    err[i] = 0.0;
    return;
  }
  const double gaa = g[a * 64 + a], gbb = g[b * 64 + b];
  const double d2 = gaa + gbb - 2.0 * g[a * 64 + b];
  // K k-steps: K roundings of k-step sums, random in sign
  const double ksteps = ceil(double(seg_end[s] - seg_lo[s]) / kKStep);
  double e = ksteps > 0.0 ? kErrCoef * (gaa + gbb) / sqrt(ksteps) : 0.0;
  if (!(d2 >= -e) || !(e < __builtin_inf())) e = __builtin_inf();
  segsq[i] = d2 > 0.0 ? d2 : 0.0;
  err[i] = e;
}

// D[a][b] = Σ_s fl32(sqrt(segsq[s][a][b])) in key order (fp32, as
// pairdist_finish_kernel and the reference's `distance += torch.dist`),
// D[a][a] = +inf; ill[a][b] = 1 when the keys' error bounds could move
// the distance by more than tol·D (or it is not finite).  Per key the
// random part δ = err moves d = sqrt(d²) by at most min(δ / 2d, sqrt(δ));
// the keys' parts are independent (summed in quadrature); the part
// proportional to d² moves D by kErrBias / 2 · D.
__global__ __launch_bounds__(256) void gram_finish_kernel(
    const double *__restrict__ segsq, const double *__restrict__ err, int n,
    int nseg, double tol, float *__restrict__ D, uint32_t *__restrict__ ill) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= n * n) return;
  if (q / n == q % n) {
    D[q] = __builtin_inff();
    ill[q] = 0u;
    return;
  }
  float dist = 0.0f;
  double var = 0.0;
  bool inf = false;
  for (int s = 0; s < nseg; ++s) {
    const double d2 = segsq[int64_t(s) * n * n + q];
    const double e = err[int64_t(s) * n * n + q];
    const double d = sqrt(d2);
    dist = add_rn(dist, float(d));
    inf = inf || !(e < __builtin_inf());
    if (e > 0.0) {
      const double m = d2 > 0.0 ? fmin(e / (2.0 * d), sqrt(e)) : sqrt(e);
      var += m * m;
    }
  }
  D[q] = dist;
  const double bound = sqrt(var) + 0.5 * kErrBias * double(dist);
  ill[q] = (!inf && bound <= tol * double(dist) && dist < __builtin_inff())
               ? 0u : 1u;
}

struct GramPlan {
  int nt;
  int64_t w;           // main chunk length (multiple of kUnit)
  int main_chunks;     // upper bounds
  int sample_chunks;
  int main_groups;
  int sample_groups;
};

GramPlan gram_plan(int n, int64_t numel, int nseg) {
  GramPlan pl;
  pl.nt = (n + 15) / 16;
  int64_t w = (numel + kMainChunks - 1) / kMainChunks;
  w = (w + kUnit - 1) / kUnit * kUnit;
  if (w < kUnit) w = kUnit;
  if (w > kMaxW) w = kMaxW;
  pl.w = w;
  pl.main_chunks = int(numel / w) + nseg + 1;
  pl.main_groups = pl.main_chunks / kRed + nseg + 1;
  const int per_key = int((kSampleCoords + kSampleChunk - 1) / kSampleChunk);
  pl.sample_chunks = nseg * per_key;
  pl.sample_groups = nseg * ((per_key + kRed - 1) / kRed);
  return pl;
}

struct GramWs {
  int *prefix_main, *gprefix_main, *prefix_sample, *gprefix_sample, *centre;
  double *partial, *g_sample, *g_main, *red;
};

size_t gram_ws_layout(int n, int64_t numel, int nseg, void *ws, GramWs *w) {
  const GramPlan pl = gram_plan(n, numel, nseg);
  const size_t ntp = size_t(ntp_of(pl.nt));
  const size_t ints = align256(sizeof(int) * size_t(nseg + 1));
  const size_t chunks = size_t(pl.main_chunks > pl.sample_chunks
                                   ? pl.main_chunks
                                   : pl.sample_chunks);
  const size_t groups = size_t(pl.main_groups > pl.sample_groups
                                   ? pl.main_groups
                                   : pl.sample_groups);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align256(bytes);
    return static_cast<char *>(ws) + o;
  };
  char *p_pm = take(ints), *p_gm = take(ints), *p_ps = take(ints),
       *p_gs = take(ints), *p_c = take(256),
       *p_gsm = take(sizeof(double) * 64 * 64),
       *p_gmn = take(sizeof(double) * 64 * 64 * size_t(nseg)),
       *p_red = take(sizeof(double) * groups * ntp * 256),
       *p_part = take(sizeof(double) * chunks * ntp * 256);
  if (w) {
    w->prefix_main = reinterpret_cast<int *>(p_pm);
    w->gprefix_main = reinterpret_cast<int *>(p_gm);
    w->prefix_sample = reinterpret_cast<int *>(p_ps);
    w->gprefix_sample = reinterpret_cast<int *>(p_gs);
    w->centre = reinterpret_cast<int *>(p_c);
    w->g_sample = reinterpret_cast<double *>(p_gsm);
    w->g_main = reinterpret_cast<double *>(p_gmn);
    w->red = reinterpret_cast<double *>(p_red);
    w->partial = reinterpret_cast<double *>(p_part);
  }
  return off;
}

template <int NT>
void gram_launch(const float *const *tab, int64_t ss, int n,
                 const int64_t *seg_lo, const int64_t *seg_end, int nseg,
                 const GramPlan &pl, const GramWs &w, double *segsq,
                 double *err, hipStream_t st) {
  constexpr int NTP = ntp_of(NT);
  // 1. the centre: Gram of the first kSampleCoords of every key, raw
  hipLaunchKernelGGL(gram_prefix_kernel, dim3(1), dim3(1), 0, st, seg_lo,
                     seg_end, nseg, kSampleChunk, kSampleCoords,
                     w.prefix_sample, w.gprefix_sample);
  hipLaunchKernelGGL((gram_chunk_kernel<NT, false>),
                     dim3(unsigned(pl.sample_chunks)), dim3(kBlk), 0, st,
                     tab, ss, n, seg_lo, seg_end, nseg, w.prefix_sample,
                     kSampleChunk, kSampleCoords,
                     static_cast<const int *>(nullptr), w.partial);
  hipLaunchKernelGGL((gram_reduce1_kernel<NT>),
                     dim3(unsigned(pl.sample_groups), unsigned(NTP)),
                     dim3(256), 0, st, w.partial, w.prefix_sample,
                     w.gprefix_sample, nseg, w.red);
  hipLaunchKernelGGL((gram_reduce2_kernel<NT>), dim3(1, unsigned(NTP)),
                     dim3(256), 0, st, w.red, w.gprefix_sample, nseg, 1,
                     w.g_sample);
  hipLaunchKernelGGL(gram_centre_kernel, dim3(1), dim3(256), 0, st,
                     w.g_sample, n, w.centre);
  // 2. the centred Gram of every key
  hipLaunchKernelGGL(gram_prefix_kernel, dim3(1), dim3(1), 0, st, seg_lo,
                     seg_end, nseg, pl.w, int64_t(0), w.prefix_main,
                     w.gprefix_main);
  hipLaunchKernelGGL((gram_chunk_kernel<NT, true>),
                     dim3(unsigned(pl.main_chunks)), dim3(kBlk), 0, st, tab,
                     ss, n, seg_lo, seg_end, nseg, w.prefix_main, pl.w,
                     int64_t(0), static_cast<const int *>(w.centre),
                     w.partial);
  hipLaunchKernelGGL((gram_reduce1_kernel<NT>),
                     dim3(unsigned(pl.main_groups), unsigned(NTP)),
                     dim3(256), 0, st, w.partial, w.prefix_main,
                     w.gprefix_main, nseg, w.red);
  hipLaunchKernelGGL((gram_reduce2_kernel<NT>),
                     dim3(unsigned(nseg), unsigned(NTP)), dim3(256), 0, st,
                     w.red, w.gprefix_main, nseg, 0, w.g_main);
  const int64_t tot = int64_t(nseg) * n * n;
  hipLaunchKernelGGL(gram_segsq_kernel, dim3(unsigned((tot + 255) / 256)),
                     dim3(256), 0, st, w.g_main, seg_lo, seg_end, n, nseg,
                     segsq, err);
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" size_t fsagg_pairgram_workspace_bytes(int n, int64_t numel,
                                                 int nseg) {
  if (n < 2 || n > 16 * kGramMaxTiles || nseg < 1 || numel < 0) return 0;
  return gram_ws_layout(n, numel, nseg, nullptr, nullptr);
}

extern "C" int fsagg_pairgram_rows_segsq_f32(const fsagg_rows *rows,
                                             const int64_t *seg_lo,
                                             const int64_t *seg_end,
                                             int64_t numel, double *segsq,
                                             double *err, void *workspace,
                                             size_t workspace_bytes,
                                             fsagg_stream_t stream) {
  if (!rows || !rows->tab || !seg_lo || !seg_end || !segsq || !err ||
      rows->n < 2 || rows->n > 16 * kGramMaxTiles || rows->nseg < 1 ||
      numel < 0 || (rows->ss != 0 && rows->ss < rows->n)) {
    set_error("fsagg_pairgram_rows_segsq_f32: invalid argument (n must be "
              "2..%d)", 16 * kGramMaxTiles);
    return FSAGG_EINVAL;
  }
  const int n = rows->n, nseg = rows->nseg;
  const size_t need = gram_ws_layout(n, numel, nseg, nullptr, nullptr);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_pairgram_rows_segsq_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  const GramPlan pl = gram_plan(n, numel, nseg);
  GramWs w;
  gram_ws_layout(n, numel, nseg, workspace, &w);
  hipStream_t st = as_stream(stream);
  switch (pl.nt) {
    case 1: gram_launch<1>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, err, st); break;
    case 2: gram_launch<2>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, err, st); break;
    case 3: gram_launch<3>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                           w, segsq, err, st); break;
    default: gram_launch<4>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl,
                            w, segsq, err, st); break;
  }
  return check_launch("fsagg_pairgram_rows_segsq_f32");
}

extern "C" int fsagg_pairgram_finish_f32(const double *segsq,
                                         const double *err, int n, int nseg,
                                         double tol, float *D, uint32_t *ill,
                                         fsagg_stream_t stream) {
  if (!segsq || !err || !D || !ill || n < 2 || nseg < 1 || !(tol >= 0.0)) {
    set_error("fsagg_pairgram_finish_f32: invalid argument (n=%d nseg=%d)",
              n, nseg);
    return FSAGG_EINVAL;
  }
  hipLaunchKernelGGL(gram_finish_kernel,
                     dim3(unsigned((int64_t(n) * n + 255) / 256)), dim3(256),
                     0, as_stream(stream), segsq, err, n, nseg, tol, D, ill);
  return check_launch("fsagg_pairgram_finish_f32");
}
