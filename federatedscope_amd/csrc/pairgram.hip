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
//   v_dot2c_f32_bf16 each; x − h holds at most 16 significant bits and
//   x − h − m at most 8, so l takes the rest exactly).  The six limb
//   products of weight >= 2^-16 (hh, hm, mh, hl, lh, mm) are exact in the
//   MFMA; the dropped ones (ml, lm, ll) are <= 2.02·2^-24 of |x_a·x_b|.
//   Each k-step's six products of a tile pair are
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
//   Every per-key d² leaves with a worst-case error bound err (limb
//   products, the MFMA's rounding, fp64 sums, centring, underflow: see
//   kCoefLimb below); fsagg_pairgram_finish_f32 sums those into a bound B
//   on every pair's D, which the caller certifies its Krum selection with
//   (core/aggregators/_engine.certified_selection), recomputing D on the
//   VALU kernel when the score gaps do not clear it.  Non-finite pairs are
//   flagged and recomputed on the VALU kernel (its ±inf / NaN semantics).
//
// Work: a workgroup of 4 waves per chunk of one key; wave v takes the
// chunk's k-steps v, v + 4, ... (n <= 112; above, the tile-split
// workgroups of gram_block8_kernel).  The chunk's rows stream through LDS in
// stages (global_load_lds_dwordx4, 512-B runs per row: see kGramStaged) and
// are read back in MFMA fragment order (lane l: client 16t + (l & 15);
// fragment slots 0-3 = coordinates 4(l>>4) .. +3 and slots 4-7 =
// 16 + 4(l>>4) .. +3 of the k-step — any permutation of k is a valid
// contraction as long as both operands use it); every value is read from
// HBM once.
#include <atomic>
#include <type_traits>

#include "common.h"

namespace fsagg {
namespace {

typedef short frag8 __attribute__((ext_vector_type(8)));     // 8 bf16
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kGramMaxTiles = 16;         // n <= 256
constexpr int kPlaneTiles = 13;           // PG(2, 3): the lines' limit
constexpr int kFullTiles = 4;             // one workgroup forms every pair
constexpr int kKStep = 32;                // coordinates per MFMA k-step
constexpr int kWaves = 4;                 // waves per workgroup (chunk)
constexpr int kBlk = kWaves * kWave;
constexpr int64_t kUnit = kKStep * kWaves;  // chunk lengths: multiples
constexpr int kRed = 32;                  // chunks per first-level sum
constexpr int kMainChunks = 1024;         // ~2 rounds at 2 blocks per CU
constexpr int kOneMaxTiles = 7;           // one workgroup up to 112 clients
constexpr int64_t kMaxW = 16384;          // chunk length cap (LDS centre)
constexpr int64_t kSampleCoords = 2048;   // per key, for the centre choice
constexpr int64_t kSampleChunk = 512;
constexpr int kLineBlocks = 8192;         // n > 64: ~workgroups per pass

// Worst-case error bound of a key's d²(a, b) (segsq_pair; DESIGN
// §3.3 derives each term).  u = 2^-24; S = sqrt(G'aa) + sqrt(G'bb), so
// Σ_p |x'_a[p]·x'_b[p]| <= sqrt(G'aa·G'bb) and G'aa + G'bb + 2·sqrt(G'aa·G'bb)
// = S² bound every Gram entry's magnitude sum (Cauchy-Schwarz):
// * limbs: x = h + m + l EXACTLY (8 + 8 + 8 significant bits of a 24-bit
//   significand, the residuals' signs absorbing the rounding), so the only
//   product error is the three dropped limb products ml, lm, ll:
//   <= (2·2^-24 + 2^-32)·(1 + 2^-8)²·|x·y|            -> kCoefLimb · u · S²
// * MFMA accumulation: v_mfma_f32_16x16x32_bf16 aligns its 32 exact
//   products and C to the largest and truncates what lies below a window
//   of about 26 bits under its leading bit, then rounds once
//   (tools/probe/mfma_numerics.py, profiles/r04/mfma_numerics.jsonl and
//   mfma_window.jsonl: 31 same-sign terms below 2^-27 of the largest vanish
//   whole; the worst error over every family probed is 7.5·u·Σ|terms|, and
//   9.4·u·max|term| where the terms cancel): each of the 33 terms loses
//   < 2^-26·max|term|, the rounding <= u·|result|, so the error is
//   <= (33·2^-26/u)·u·max|term| + u·|result| <= 9.25·u·Σ|terms| per MFMA
//   (bound used: 10); over the chain mm, hl, lh, hm, mh, hh those sums
//   total <= 1.035·Σ|x·y|                        -> 1.035·kMfmaRound
// * fp64: the K k-step sums, four waves and two reduction levels add
//   <= (K + 1024) · 2^-53 relative                     -> (K + 1024)·2^-29
// * centring x' = fl32(x − x_c) perturbs the rows by <= u·|x'|: d² moves by
//   <= 2u·d·S + u²·S²
// * underflow (limbs or products below 2^-126, flushed or subnormal):
//   <= 2^-126 · (12·sqrt(P)·S + 800·K) absolute
constexpr double kU = 5.9604644775390625e-08;   // 2^-24
constexpr double kCoefLimb = 2.02;
constexpr double kMfmaRound = 10.0;
constexpr double kMfmaChain = 1.035;
constexpr double kTiny = 1.1754943508222875e-38;  // 2^-126

constexpr int ntp_of(int nt) { return nt * (nt + 1) / 2; }

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Per-pass plan (device workspace ints): chunk q of key s covers
// [seg_lo[s] + q·w, min(seg_lo[s] + (q+1)·w, cap_s)), cap_s = seg_end[s]
// (or seg_lo[s] + cap for the sample pass); its chunks are prefix[s] ..
// prefix[s+1] − 1 and its first-level groups (kRed chunks each)
// gprefix[s] .. gprefix[s+1] − 1.
struct GramCtl {
  int *prefix;      // [nseg + 1]
  int *gprefix;     // [nseg + 1]
  int desync;       // A/B: main-pass start offset (fsagg_pairgram_set_desync)
};

// One wave: lane l takes keys l, l + 64, ...; the chunk and group counts
// are prefix-summed across the wave (one 64-bit division per lane instead
// of nseg in a row: 6.1 us for both plans from one thread at C4).
__device__ void plan_pass(const int64_t *__restrict__ seg_lo,
                          const int64_t *__restrict__ seg_end, int nseg,
                          int64_t w, int64_t cap, const GramCtl &c) {
  const int lane = int(threadIdx.x) & (kWave - 1);
  if (lane == 0) {
    c.prefix[0] = 0;
    c.gprefix[0] = 0;
  }
  int base = 0, gbase = 0;
  for (int s0 = 0; s0 < nseg; s0 += kWave) {
    const int s = s0 + lane;
    int k = 0, g = 0;
    if (s < nseg) {
      int64_t len = seg_end[s] - seg_lo[s];
      if (cap > 0 && len > cap) len = cap;
      if (len < 0) len = 0;
      k = int((len + w - 1) / w);
      g = (k + kRed - 1) / kRed;
    }
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int kk = __shfl_up(k, d, kWave), gg = __shfl_up(g, d, kWave);
      if (lane >= d) {
        k += kk;
        g += gg;
      }
    }
    if (s < nseg) {
      c.prefix[s + 1] = base + k;
      c.gprefix[s + 1] = gbase + g;
    }
    base += __shfl(k, kWave - 1, kWave);
    gbase += __shfl(g, kWave - 1, kWave);
  }
}

// Both passes' plans in one launch: wave 0 the sample pass, wave 1 the
// main pass.
__global__ __launch_bounds__(2 * kWave) void gram_prefix_kernel(
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, int64_t w_sample, int64_t cap_sample, int64_t w_main,
    GramCtl cs, GramCtl cm, unsigned *__restrict__ tickets, int ntickets) {
  // the fused tail's arrival tickets (vector stores: per-lane addresses)
  for (int i = int(threadIdx.x); i < ntickets; i += 2 * kWave)
    __hip_atomic_store(tickets + i, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kWave)
    plan_pass(seg_lo, seg_end, nseg, w_sample, cap_sample, cs);
  else
    plan_pass(seg_lo, seg_end, nseg, w_main, 0, cm);
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

// Split 8 fp32 into three packed bf16 limbs: x = h + m + l exactly (for
// |x| >= 2^-102, where l stays a normal bf16), residuals of both signs.
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
__device__ __forceinline__ void kstep_split_c(const float (&xb)[NT][8],
                                              const float (&cb)[8],
                                              const Neg &k, Frags<NT> &f) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = CENTRED ? xb[t][j] - cb[j] : xb[t][j];
    split3(x, k, f.h[t], f.m[t], f.l[t]);
  }
}

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
  kstep_split_c<NT, CENTRED>(xb, cb, k, f);
}

// n > 64 (T > 4 tiles of 16 clients): every workgroup forms every pair of
// its NT tiles, and the tile sets are the lines of a finite projective
// plane, which hold every pair of points exactly once — PG(2, 3): 13 points,
// 13 lines of 4 (T <= 13, the difference set {0, 1, 3, 9} mod 13); PG(2, 2)
// (Fano): 7 points, 7 lines of 3 (T <= 7, {0, 1, 3} mod 7).  Each tile is
// loaded and split 4 (3) times per chunk, not once per super-tile pair; a
// point's diagonal block is stored by the line it generates.  Points >= T
// are absent (their rows clamp to the last client, their pairs are not
// stored).  Lines sorted, so t < u within a line maps to tile t < tile u.
__constant__ int8_t kPlane13[13][4] = {
    {0, 1, 3, 9},  {1, 2, 4, 10}, {2, 3, 5, 11}, {3, 4, 6, 12}, {0, 4, 5, 7},
    {1, 5, 6, 8},  {2, 6, 7, 9},  {3, 7, 8, 10}, {4, 8, 9, 11}, {5, 9, 10, 12},
    {0, 6, 10, 11}, {1, 7, 11, 12}, {0, 2, 8, 12}};
__constant__ int8_t kPlane7[7][3] = {{0, 1, 3}, {1, 2, 4}, {2, 3, 5},
                                     {3, 4, 6}, {0, 4, 5}, {1, 5, 6},
                                     {0, 2, 6}};

// index of tile pair (t, u), t <= u, among the T(T+1)/2 (tp_tiles' order)
__device__ __forceinline__ int pair_index(int t, int u, int T) {
  return t * T - (t * (t - 1)) / 2 + (u - t);
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

// d²(a, b) of one key from its Gram entries G'aa, G'bb, G'ab and its
// worst-case error bound (the terms at kCoefLimb); +inf when d² came out
// negative beyond that bound or is not finite (the pair is recomputed).
__device__ __forceinline__ void segsq_pair(double gaa, double gbb, double gab,
                                           bool same, int64_t len,
                                           double &d2o, double &eo) {
  if (same) {
    d2o = 0.0;
    eo = 0.0;
    return;
  }
  const double d2 = gaa + gbb - 2.0 * gab;
  const double K = double((len + kKStep - 1) / kKStep);
  // S from the computed diagonal, inflated for its own error (the relative
  // bound below is < 1e-5 of it)
  const double S = (sqrt(fmax(gaa, 0.0)) + sqrt(fmax(gbb, 0.0))) *
                   (1.0 + 1e-5);
  const double S2 = S * S;
  const double coef = kCoefLimb + kMfmaChain * kMfmaRound +
                      (K + 1024.0) * 0x1p-29 + 4.0 * 0x1p-29;
  const double e_gram = coef * kU * S2;
  const double d_up = fmin(S, sqrt(fmax(d2, 0.0) + e_gram));
  const double e_centre = 2.0 * kU * d_up * S + kU * kU * S2;
  const double e_tiny = kTiny * (12.0 * sqrt(double(len)) * S + 800.0 * K);
  double e = len > 0 ? (e_gram + e_centre + e_tiny) * (1.0 + 1e-9) : 0.0;
  if (!(d2 >= -e) || !(e < __builtin_inf())) e = __builtin_inf();
  d2o = d2 > 0.0 ? d2 : 0.0;
  eo = e;
}

// D[q] = Σ_s fl32(sqrt(segsq[s][q])) in key order (fp32, as
// pairdist_finish_kernel and the reference's `distance += torch.dist`),
// D[a][a] = +inf; ill[q] = 1 unless the keys' distances are certified to tol
// of the exact ones: Σ_s δ_s <= tol · Σ_s d_s, where δ_s is the worst move
// of d = sqrt(d²) over the d² interval [d² − e, d² + e] (at most
// e / (sqrt(d²) + sqrt(d² − e)) and sqrt(e)), summed linearly over the keys.
// D itself is the reference's fp32 formation of those per-key distances;
// D64 (optional) the same sum in fp64, Σ_s sqrt(d²_s), which B bounds
// without D's own fp32 rounding.
__device__ __forceinline__ void finish_pair(int q, const double *segsq,
                                            const double *err, int n,
                                            int nseg, double tol, float *D,
                                            uint32_t *ill, float *B,
                                            double *D64) {
  if (q / n == q % n) {
    D[q] = __builtin_inff();
    ill[q] = 0u;
    if (B) B[q] = 0.0f;
    if (D64) D64[q] = __builtin_inf();
    return;
  }
  float dist = 0.0f;
  double sum_d = 0.0, bound = 0.0;
  bool inf = false;
  for (int s = 0; s < nseg; ++s) {
    const int64_t at = int64_t(s) * n * n + q;
    const double d2 = segsq[at];
    const double e = err[at];
    const double d = sqrt(d2);
    dist = add_rn(dist, float(d));
    sum_d += d;
    inf = inf || !(e < __builtin_inf());
    if (e > 0.0) {
      const double up = sqrt(d2 + e) - d;
      const double dn = d - sqrt(fmax(d2 - e, 0.0));
      bound += fmax(up, dn);
    }
  }
  D[q] = dist;
  if (D64) D64[q] = sum_d;
  // tol = +inf: only non-finite pairs are flagged (inf · 0 is NaN, so the
  // relative test is skipped rather than evaluated)
  const bool close = !(tol < __builtin_inf()) || bound <= tol * sum_d;
  ill[q] = (!inf && close && dist < __builtin_inff()) ? 0u : 1u;
  // the bound on |D − the exact per-key distances' sum|, rounded up to fp32
  if (B) B[q] = inf ? __builtin_inff() : __double2float_ru(bound);
}

// finish_pair of pair q, stored at q and at its mirror q2 (the key sums
// are symmetric, so both entries are the same values): the keys' d² and
// bounds are loaded eight keys at a time (a loop of dependent loads costs
// the fused tail's last workgroups one memory round trip per key — they
// read other workgroups' fresh stores, which no cache holds); the
// arithmetic is finish_pair's, in the same order.
__device__ __forceinline__ void finish_pair_sym(int q, int q2,
                                                const double *segsq,
                                                const double *err, int n,
                                                int nseg, double tol,
                                                float *D, uint32_t *ill,
                                                float *B, double *D64) {
  if (q / n == q % n) {
    finish_pair(q, segsq, err, n, nseg, tol, D, ill, B, D64);
    return;
  }
  const int64_t nn = int64_t(n) * n;
  float dist = 0.0f;
  double sum_d = 0.0, bound = 0.0;
  bool inf = false;
  for (int s0 = 0; s0 < nseg; s0 += 8) {
    double d2v[8], ev[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t at = int64_t(min(s0 + j, nseg - 1)) * nn + q;
      d2v[j] = segsq[at];
      ev[j] = err[at];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (s0 + j >= nseg) break;
      const double d2 = d2v[j], e = ev[j];
      const double d = sqrt(d2);
      dist = add_rn(dist, float(d));
      sum_d += d;
      inf = inf || !(e < __builtin_inf());
      if (e > 0.0) {
        const double up = sqrt(d2 + e) - d;
        const double dn = d - sqrt(fmax(d2 - e, 0.0));
        bound += fmax(up, dn);
      }
    }
  }
  const bool close = !(tol < __builtin_inf()) || bound <= tol * sum_d;
  const uint32_t flag = (!inf && close && dist < __builtin_inff()) ? 0u : 1u;
  const float bq = inf ? __builtin_inff() : __double2float_ru(bound);
  D[q] = dist;
  ill[q] = flag;
  if (B) B[q] = bq;
  if (D64) D64[q] = sum_d;
  if (q2 != q) {
    D[q2] = dist;
    ill[q2] = flag;
    if (B) B[q2] = bq;
    if (D64) D64[q2] = sum_d;
  }
}

// Staged loads (kGramStaged): the chunk streams through LDS in stages of
// kStage coordinates.  Each stage holds every row's kStage·4 = 512 B — the
// 16·NT tile rows, then the centre's — written by global_load_lds_dwordx4
// (one wave-instruction = 1 KiB = two rows) and read back in MFMA fragment
// order.  A row's 512 B leave in one instruction: 50 rows that all start at
// one offset within a 2 MiB page (separately allocated tensors) are read as
// 512-B runs, not as the 128-B pieces each wave's own k-step loads take.
// The LDS image is lane-linear per instruction, so the bank swizzle goes on
// the SOURCE address: row r's 16-B chunk c sits in slot c ^ (r & 15), and
// the 16 lanes of a fragment read (rows 16t .. 16t + 15, one chunk) hit 16
// distinct bank quads.
#ifdef FSAGG_GRAM_REGS   // probe builds only (tools/probe): the register path
constexpr bool kGramStaged = false;
#else
constexpr bool kGramStaged = true;
#endif
constexpr int kStage = kKStep * kWaves;          // 128 coordinates
constexpr int kStageRowBytes = kStage * 4;       // 512 B

template <int NT, bool CENTRED>
constexpr int stage_rows() { return 16 * NT + (CENTRED ? 1 : 0); }
template <int NT, bool CENTRED>
constexpr int stage_insts() { return (stage_rows<NT, CENTRED>() + 1) / 2; }
// one stage buffer (rows rounded up to the instructions' row pairs)
template <int NT, bool CENTRED>
constexpr int stage_bytes() {
  return 2 * stage_insts<NT, CENTRED>() * kStageRowBytes;
}
template <int NT, bool CENTRED>
constexpr int chunk_smem() {
  constexpr int red = 2 * ntp_of(NT) * 4 * kWave * 8;    // two waves' sums
  constexpr int stg = kGramStaged ? 2 * stage_bytes<NT, CENTRED>()
                                  : int(kMaxW) * 4;       // or the centre
  return red > stg ? red : stg;
}

// The 8 values of lane (row rr, group g) for k-step ks of a stage buffer.
__device__ __forceinline__ void stage_read8(const char *buf, int rr, int ks,
                                            int g, float (&v)[8]) {
  typedef __attribute__((address_space(3))) const f32x4 lds_f32x4;
  const int c0 = 8 * ks + g, c1 = c0 + 4;
  const char *r = buf + rr * kStageRowBytes;
  const f32x4 x = *(lds_f32x4 *)(uintptr_t)(r + 16 * (c0 ^ (rr & 15)));
  const f32x4 y = *(lds_f32x4 *)(uintptr_t)(r + 16 * (c1 ^ (rr & 15)));
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

// Compact stages (!LINES, the default forms): the chunk's n client rows
// only — row j of the stage is client j, the centre is read from its own
// row (it is one of the clients), rows past n are never staged (their
// fragment lanes read row n − 1, an LDS broadcast) — and NBUF buffers, so
// NBUF − 1 stages are in flight while one is computed.  A stage of
// ⌈n/2⌉ 1-KiB instructions; MAXI bounds it (the static LDS): at two
// workgroups per CU (NT <= 4) three buffers fit 80 KiB up to 52 clients,
// at one per CU (5 <= NT <= 7) 160 KiB up to 104.  Every wave issues the
// same 2·NT loads per stage (instructions past the last one repeat it: the
// same bytes into the same LDS slot, from L2), so `s_waitcnt vmcnt` can
// name the loads of the stages still allowed in flight.
template <int NT>
constexpr int compact_maxi3() {
  return NT <= kFullTiles ? (8 * NT < 26 ? 8 * NT : 26)
                          : (8 * NT < 52 ? 8 * NT : 52);
}

// s_waitcnt vmcnt(k · loads) for the k stages still allowed in flight
template <int LOADS>
__device__ __forceinline__ void wait_stage(int ahead) {
  if (ahead <= 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else if (ahead == 1) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(LOADS)
                 : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(
                     2 * LOADS)
                 : "memory");
  }
}

// One workgroup (4 waves) per chunk (its NT tiles are all the tiles: n <=
// 64 at two workgroups per CU, and up to kOneMaxTiles tiles at one per CU
// with the accumulators spread over VGPRs and AGPRs) or per chunk and plane
// line (LINES, the A/B setting 0 for n > 64).  partial[chunk][tp]
// [reg][lane] (fp64, tp over the T(T+1)/2 tile pairs): the chunk's
// (centred) Gram blocks in MFMA C-layout (row 4(lane>>4) + reg of tile t,
// column lane & 15 of tile u).  !CENTRED: raw values (sample).  The rows
// stream through LDS stages (kGramStaged, above; wave v takes k-step v of
// every stage); without it each wave loads its own k-steps straight into
// registers and the centre's values of the chunk are staged in LDS once.
// LINES: block b takes chunk 8·(k / lines) + b % 8 and line k % lines
// (k = b / 8): blocks b and b + 8 share an XCD, so one chunk's workgroups
// run on one XCD together and read its rows from that XCD's L2 after the
// first.
// cache policy of the stage loads: NT (non-temporal, gfx950 CPol bit 1) —
// the rows are read once.  Interleaved A/B of the whole chain against plain
// loads (stages 4; profiles/r06/gram_nt_default_ab.jsonl, medians of 8
// rounds): n = 40 0.2370 against 0.2458 ms, 50 0.3101 / 0.3112, 64
// 0.3508 / 0.3519, 66 0.478 / 0.483, 100 0.880 / 0.887, 112 0.885 /
// 0.897; D64 identical
constexpr int kStageNT = 2;

template <int NT, bool CENTRED>
constexpr int compact_smem(int maxi, int nbuf) {
  constexpr int red = 2 * ntp_of(NT) * 4 * kWave * 8;
  return red > nbuf * maxi * 1024 ? red : nbuf * maxi * 1024;
}

template <int NT, bool CENTRED, bool LINES, int MAXI = 0, int NBUF = 2,
          bool EARLY = false, bool PRIO = false, int AUX = kStageNT>
__global__ __launch_bounds__(kBlk, (NT > kFullTiles ? 1 : 2))
void gram_chunk_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n, int T,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, GramCtl ctl, int64_t w, int64_t cap,
    const int *__restrict__ centre, double *__restrict__ partial) {
  static_assert(!LINES || NT == 3 || NT == 4, "plane lines hold 3 or 4");
  static_assert(MAXI == 0 || (!LINES && (NBUF == 2 || NBUF == 3)),
                "compact stages: MAXI instructions, 2 or 3 buffers");
  constexpr int NTP = ntp_of(NT);
  constexpr int kLines = NT == 4 ? 13 : 7;
  const int *__restrict__ prefix = ctl.prefix;
  constexpr int kSmem = MAXI == 0 || !kGramStaged
                            ? chunk_smem<NT, CENTRED>()
                            : compact_smem<NT, CENTRED>(MAXI, NBUF);
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  double(*red)[NTP * 4][kWave] =
      reinterpret_cast<double(*)[NTP * 4][kWave]>(smem);
  float *cs = reinterpret_cast<float *>(smem);
  int chunk = blockIdx.x, line = 0;
  if constexpr (LINES) {
    const int k = int(blockIdx.x >> 3);
    chunk = (k / kLines) * 8 + int(blockIdx.x & 7);
    line = k % kLines;
  }
  // global tile of local tile lt
  auto gtile = [&](int lt) {
    return LINES ? int(NT == 4 ? kPlane13[line][lt] : kPlane7[line][lt])
                 : lt;
  };
  if (chunk >= prefix[nseg]) return;   // whole workgroup
  if (CENTRED && ctl.desync > 3) {
    const int sel = ctl.desync & 3;
    const unsigned bit = sel == 1 ? blockIdx.x : blockIdx.x >> (sel + 6);
    if (bit & 1u)
      for (int i = 0; i < (ctl.desync >> 2); ++i) __builtin_amdgcn_s_sleep(8);
  }
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
    const int j = 16 * gtile(t) + (lane & 15);
    row[t] = rows[j < n ? j : n - 1];
  }
  const float *crow = CENTRED ? rows[*centre] : nullptr;

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
  if (CENTRED) ok = ok && al16(crow + c0);
  const bool vec = __all(ok);
  int i = wv;   // this wave's next k-step: wv, wv + 4, ...
  if constexpr (kGramStaged && MAXI > 0) {
    const int nstage = vec ? int(len / kStage) : 0;
    if (nstage > 0) {
      // this wave's load instructions k = wv, wv + 4, ... (clamped to the
      // last, NI − 1): client rows 2k (lanes 0-31) and 2k + 1 (lanes
      // 32-63), each lane one 16-B chunk, its source swizzled (chunk
      // (lane & 31) ^ (row & 15))
      constexpr int MY = 2 * NT;
      const int NI = (n + 1) >> 1;
      const int sb = NI * 2 * kStageRowBytes;
      const float *src[MY];
      int dst[MY];
#pragma unroll
      for (int m = 0; m < MY; ++m) {
        const int k = min(wv + kWaves * m, NI - 1);
        const int rr = 2 * k + (lane >> 5);
        src[m] = rows[rr < n ? rr : n - 1] + c0 + 4 * ((lane & 31) ^ (rr & 15));
        dst[m] = k * 2 * kStageRowBytes;
      }
      auto issue = [&](int st) {
        char *buf = smem + (st % NBUF) * sb;
#pragma unroll
        for (int m = 0; m < MY; ++m)
          __builtin_amdgcn_global_load_lds(
              (__attribute__((address_space(1))) void *)(src[m] + st * kStage),
              (__attribute__((address_space(3))) void *)(uintptr_t)(buf +
                                                                   dst[m]),
              16, 0, AUX);
      };
      // the rows this lane's fragments read: client 16t + (lane & 15), past
      // n the last client (never stored); the centre's own row
      int rrow[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int j = 16 * t + (lane & 15);
        rrow[t] = j < n ? j : n - 1;
      }
      const int crr = CENTRED ? *centre : 0;
#pragma unroll
      for (int p = 0; p < NBUF - (EARLY ? 0 : 1); ++p)
        if (p < nstage) issue(p);
      for (int st = 0; st < nstage; ++st) {
        if constexpr (EARLY) {
          // early release: NBUF stages in flight while one is computed.
          // Stage st has landed (this wave's loads: vmcnt, the stages
          // issued after it may stay in flight; every wave's: the
          // barrier); its fragments go to registers, and once every wave
          // has read them (the second barrier) the buffer takes stage
          // st + NBUF — the compute below runs from registers, so the
          // buffer need not sit idle under it (Little's law: the bytes in
          // flight per CU set the bandwidth at ~5 µs loaded latency)
          const int ahead = min(nstage - 1 - st, NBUF - 1);
          wait_stage<MY>(ahead);
          const char *buf = smem + (st % NBUF) * sb;
          float xb[NT][8], cb[8];
#pragma unroll
          for (int t = 0; t < NT; ++t) stage_read8(buf, rrow[t], wv, g, xb[t]);
          if (CENTRED) stage_read8(buf, crr, wv, g, cb);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          if (st + NBUF < nstage) issue(st + NBUF);
          Frags<NT> f;
          kstep_split_c<NT, CENTRED>(xb, cb, kn, f);
          kstep_mfma<NT>(f, acc);
          continue;
        }
        // stage st's loads have landed (this wave's: vmcnt; every wave's:
        // the barrier), every wave is done reading stage st − 1, whose
        // buffer the next issue overwrites
        const int ahead = min(nstage - 1 - st, NBUF - 2);
        wait_stage<MY>(ahead);
        if (st + NBUF - 1 < nstage) issue(st + NBUF - 1);
        const char *buf = smem + (st % NBUF) * sb;
        float xb[NT][8], cb[8];
#pragma unroll
        for (int t = 0; t < NT; ++t) stage_read8(buf, rrow[t], wv, g, xb[t]);
        if (CENTRED) stage_read8(buf, crr, wv, g, cb);
        Frags<NT> f;
        kstep_split_c<NT, CENTRED>(xb, cb, kn, f);
        // A/B (PRIO): the MFMA cluster at priority 1 (CDNA guide T5)
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
        kstep_mfma<NT>(f, acc);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
      }
      i = nstage * kWaves + wv;
      // the stage buffers are free again (the tail reads global memory)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  } else if constexpr (kGramStaged) {
    const int nstage = vec ? int(len / kStage) : 0;
    if (nstage > 0) {
      // this wave's load instructions k = wv, wv + 4, ... of every stage:
      // rows 2k (lanes 0-31) and 2k + 1 (lanes 32-63), each lane one 16-B
      // chunk, its source swizzled (chunk (lane & 31) ^ (row & 15))
      constexpr int NI = stage_insts<NT, CENTRED>();
      constexpr int MY = (NI + kWaves - 1) / kWaves;
      constexpr int NR = 16 * NT;
      const float *src[MY];
#pragma unroll
      for (int m = 0; m < MY; ++m) {
        const int rr = 2 * (wv + kWaves * m) + (lane >> 5);
        const int cr = 16 * gtile(rr >> 4) + (rr & 15);
        const float *rp = rr < NR ? rows[cr < n ? cr : n - 1]
                                  : (CENTRED && rr == NR ? crow
                                                         : rows[n - 1]);
        src[m] = rp + c0 + 4 * ((lane & 31) ^ (rr & 15));
      }
      auto issue = [&](int st) {
        char *buf = smem + (st & 1) * stage_bytes<NT, CENTRED>();
#pragma unroll
        for (int m = 0; m < MY; ++m) {
          const int k = wv + kWaves * m;
          if (k < NI)
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void *)(src[m] +
                                                           st * kStage),
                (__attribute__((address_space(3))) void *)(uintptr_t)(
                    buf + k * 2 * kStageRowBytes),
                16, 0, AUX);
        }
      };
      issue(0);
      for (int st = 0; st < nstage; ++st) {
        // this wave's stage-st loads have landed, every wave's (barrier),
        // and every wave is done reading stage st − 1, whose buffer the
        // next issue overwrites
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" :::
                         "memory");
        if (st + 1 < nstage) issue(st + 1);
        const char *buf = smem + (st & 1) * stage_bytes<NT, CENTRED>();
        float xb[NT][8], cb[8];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          stage_read8(buf, 16 * t + (lane & 15), wv, g, xb[t]);
        if (CENTRED) stage_read8(buf, NR, wv, g, cb);
        Frags<NT> f;
        kstep_split_c<NT, CENTRED>(xb, cb, kn, f);
        kstep_mfma<NT>(f, acc);
      }
      i = nstage * kWaves + wv;
      // the stage buffers are free again (the tail reads global memory)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  } else {
    // one buffer: the next k-step's loads go out as soon as this one is
    // split and fly while its products are formed; the first is issued
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
      const float *cr = crow + c0;
      if (al16(cr)) {
        for (int e = 4 * int(threadIdx.x); e < len; e += 4 * kBlk) {
          if (e + 4 <= len) {
            *reinterpret_cast<f32x4 *>(cs + e) =
                gld(reinterpret_cast<const f32x4 *>(cr + e));
          } else {
            for (int j = e; j < len; ++j) cs[j] = gload(cr + j);
          }
        }
      } else {
        for (int e = int(threadIdx.x); e < len; e += kBlk)
          cs[e] = gload(cr + e);
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
  }
  // unaligned rows: every k-step; aligned: the last partial stage (staged)
  // or the partial last k-step (register loads)
  const int nall = int((len + kKStep - 1) / kKStep);
  for (; i < nall; i += kWaves) {
    const int64_t k0 = c0 + int64_t(i) * kKStep;
    float xt[NT][8], cb[8];
#pragma unroll
    for (int t = 0; t < NT; ++t) ld8_tail(row[t], k0, c1, g, xt[t]);
    if (CENTRED) {
      if constexpr (kGramStaged) {
        ld8_tail(crow, k0, c1, g, cb);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = kofs(g, j);
          cb[j] = i * kKStep + o < len ? cs[i * kKStep + o] : 0.0f;
        }
      }
    }
    Frags<NT> f;
    kstep_split_c<NT, CENTRED>(xt, cb, kn, f);
    kstep_mfma<NT>(f, acc);
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
    const int ntpg = T * (T + 1) / 2;
    double *out = partial + int64_t(chunk) * ntpg * 256;
#pragma unroll
    for (int p = 0; p < NTP; ++p) {
      int t, u;
      tp_tiles(p, NT, t, u);
      const int gt = gtile(t), gu = gtile(u);
      // absent points; a diagonal block belongs to the line its point
      // generates (every point lies on NT lines)
      if (LINES && (gu >= T || (gt == gu && gt != line))) continue;
      double *o = out + int64_t(LINES ? pair_index(gt, gu, T) : p) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o[r * 64 + lane] = acc[p][r] + red[0][p * 4 + r][lane];
    }
  }
}

// Level 1, grid (groups, ntpg): group b (of key s) sums its <= kRed chunks
// in order into red[b][p][256].
__global__ __launch_bounds__(256) void gram_reduce1_kernel(
    const double *__restrict__ partial, GramCtl ctl, int nseg, int ntpg,
    double *__restrict__ red) {
  const int b = blockIdx.x, p = blockIdx.y, e = threadIdx.x;
  if (b >= ctl.gprefix[nseg]) return;
  int s = 0;
  while (ctl.gprefix[s + 1] <= b) ++s;
  const int q0 = ctl.prefix[s] + (b - ctl.gprefix[s]) * kRed;
  const int q1 = min(q0 + kRed, ctl.prefix[s + 1]);
  double v[kRed];
#pragma unroll
  for (int q = 0; q < kRed; ++q)
    v[q] = q0 + q < q1 ? partial[((int64_t(q0) + q) * ntpg + p) * 256 + e]
                       : 0.0;
  double sum = 0.0;
#pragma unroll
  for (int q = 0; q < kRed; ++q) sum += v[q];
  red[(int64_t(b) * ntpg + p) * 256 + e] = sum;
}

// Σ over items [g0, g1) of entry e of tile pair p (items = groups or chunks,
// laid out [item][ntpg][256]), in order; eight loads in flight.
__device__ __forceinline__ double sum_items(const double *__restrict__ v,
                                            int g0, int g1, int ntpg, int p,
                                            int e) {
  double s = 0.0;
  for (int b = g0; b < g1; b += 8) {
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      x[j] = b + j < g1 ? v[(int64_t(b + j) * ntpg + p) * 256 + e] : 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
  }
  return s;
}

// C-layout entry of diagonal element i of a tile (row = column = i)
__device__ __forceinline__ int diag_entry(int i) {
  return (i & 3) * 64 + 16 * (i >> 2) + i;
}

// One tile pair (t, u) of one Gram matrix from items [g0, g1): thread e's
// entry G'[16t + ia][16u + ib] into gab, and the two tiles' diagonals into
// dg[0..15] (tile t) and dg[16..31] (tile u), each summed as the (t, t) and
// (u, u) blocks sum them.
__device__ __forceinline__ double pair_block(const double *__restrict__ v,
                                             int g0, int g1, int T, int p,
                                             int t, int u, double *dg) {
  const int e = threadIdx.x, ntpg = T * (T + 1) / 2;
  const double gab = sum_items(v, g0, g1, ntpg, p, e);
  if (e < 32) {
    const int tt = e < 16 ? t : u;
    dg[e] = sum_items(v, g0, g1, ntpg, pair_index(tt, tt, T),
                      diag_entry(e & 15));
  }
  __syncthreads();
  return gab;
}

// The sample pass's Gram (every key's sample chunks, in order), per tile
// pair (grid ntpg): the distances of its 256 entries, their sums along each
// row (the rows of tile t) and each column (the rows of tile u) into
// rsum[p][32].
__global__ __launch_bounds__(256) void gram_centre_pairs_kernel(
    const double *__restrict__ partial, GramCtl ctl, int nseg, int n, int T,
    double *__restrict__ rsum) {
  __shared__ double dg[32];
  __shared__ double dd[16][17];
  const int p = blockIdx.x, e = threadIdx.x;
  int t, u;
  tp_tiles(p, T, t, u);
  const double gab = pair_block(partial, 0, ctl.prefix[nseg], T, p, t, u, dg);
  const int l = e & 63, r = e >> 6, ia = 4 * (l >> 4) + r, ib = l & 15;
  double d = 0.0;
  if (16 * t + ia < n && 16 * u + ib < n) {
    const double d2 = dg[ia] + dg[16 + ib] - 2.0 * gab;
    d = d2 > 0.0 ? sqrt(d2) : 0.0;
  }
  dd[ia][ib] = d;
  __syncthreads();
  if (e < 32) {
    double sum = 0.0;
    for (int j = 0; j < 16; ++j) sum += e < 16 ? dd[e][j] : dd[j][e - 16];
    rsum[p * 32 + e] = sum;
  }
}

// The centre: argmin_a Σ_b d(a, b) from the tile pairs' row sums (one
// workgroup; n <= 256), tiles summed in order, the first minimum wins.
__global__ __launch_bounds__(256) void gram_centre_pick_kernel(
    const double *__restrict__ rsum, int n, int T, int *__restrict__ centre) {
  __shared__ double tot[256];
  const int a = threadIdx.x;
  double sum = 0.0;
  if (a < n) {
    const int t = a >> 4, i = a & 15;
    for (int u = 0; u < T; ++u)
      sum += t <= u ? rsum[pair_index(t, u, T) * 32 + i]
                    : rsum[pair_index(u, t, T) * 32 + 16 + i];
  }
  tot[a] = sum;
  __syncthreads();
  if (a == 0) {
    int best = 0;
    for (int b = 1; b < n; ++b)
      if (tot[b] < tot[best]) best = b;
    *centre = best;
  }
}

// Per key and tile pair (grid nseg x ntpg): the pair's Gram block summed
// over the key's groups, then every entry's d² and worst-case bound
// (segsq_pair), stored at (a, b) and (b, a) — a diagonal block keeps its
// a <= b entries, so D is exactly symmetric.
__global__ __launch_bounds__(256) void gram_key_kernel(
    const double *__restrict__ red, GramCtl ctl, int n, int T,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    double *__restrict__ segsq, double *__restrict__ err) {
  __shared__ double dg[32];
  const int s = blockIdx.x, p = blockIdx.y, e = threadIdx.x;
  int t, u;
  tp_tiles(p, T, t, u);
  const double gab = pair_block(red, ctl.gprefix[s], ctl.gprefix[s + 1], T,
                                p, t, u, dg);
  const int l = e & 63, r = e >> 6, ia = 4 * (l >> 4) + r, ib = l & 15;
  const int a = 16 * t + ia, b = 16 * u + ib;
  if (a >= n || b >= n || (t == u && ia > ib)) return;
  double d2, er;
  segsq_pair(dg[ia], dg[16 + ib], gab, a == b, seg_end[s] - seg_lo[s], d2,
             er);
  const int64_t o = int64_t(s) * n * n;
  segsq[o + int64_t(a) * n + b] = d2;
  err[o + int64_t(a) * n + b] = er;
  segsq[o + int64_t(b) * n + a] = d2;
  err[o + int64_t(b) * n + a] = er;
}

// ---- Fused tail (round 6): the centre pick behind the sample pass's pair
// sums, and key + finish in one launch behind the main pass's level-1 sums.  Both
// hand results between workgroups of one launch by an arrival ticket (the
// in-launch split-K recipe of the CDNA guide, write-through form: the
// handed-off values are stored sc1, every storing wave drains its stores,
// the workgroup's barrier, one lane's relaxed agent-scope ticket add; the
// workgroup whose add comes last takes an agent-scope acquire fence and
// reads the others' stores with plain loads).
// The tickets are zeroed by gram_prefix_kernel at the head of every chain.

// A handed-off store: write-through (global_store … sc1, agent scope), so
// the hand-off needs no release fence — a release (buffer_wbl2) in each of
// the tail's 120 workgroups at C4 cost the first build ~80 µs, the
// write-backs of one XCD's L2 running one after another.
__device__ __forceinline__ void store_wt(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The drain + ticket of one workgroup whose handed-off bytes were all
// stored write-through (store_wt); true in every thread of the workgroup
// that drew the last ticket (after its acquire).
__device__ __forceinline__ bool last_arrival(unsigned *ticket,
                                             unsigned arrivals,
                                             int *flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(
        ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == arrivals - 1u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag_lds = last;
  }
  __syncthreads();
  return *flag_lds != 0;
}

// gram_centre_pairs_kernel, and the last of its ntpg workgroups picks the
// centre from every pair's row sums (gram_centre_pick_kernel's loop).
__global__ __launch_bounds__(320) void gram_centre_fused_kernel(
    const double *__restrict__ partial, GramCtl ctl, int nseg, int n, int T,
    double *__restrict__ rsum, unsigned *__restrict__ ticket,
    int *__restrict__ centre) {
  __shared__ double dg[32];
  __shared__ double dd[16][17];
  __shared__ double tot[256];
  __shared__ int flag;
  const int p = blockIdx.x, e = threadIdx.x;
  const int ntpg = T * (T + 1) / 2, nch = ctl.prefix[nseg];
  int t, u;
  tp_tiles(p, T, t, u);
  // waves 0-3 the block's entries, wave 4 the two tiles' diagonals, at the
  // same time (pair_block's sums)
  double gab = 0.0;
  if (e < 256) {
    gab = sum_items(partial, 0, nch, ntpg, p, e);
  } else if (e < 256 + 32) {
    const int q = e - 256, tt = q < 16 ? t : u;
    dg[q] = sum_items(partial, 0, nch, ntpg, pair_index(tt, tt, T),
                      diag_entry(q & 15));
  }
  __syncthreads();
  const int l = e & 63, r = (e >> 6) & 3, ia = 4 * (l >> 4) + r, ib = l & 15;
  if (e < 256) {
    double d = 0.0;
    if (16 * t + ia < n && 16 * u + ib < n) {
      const double d2 = dg[ia] + dg[16 + ib] - 2.0 * gab;
      d = d2 > 0.0 ? sqrt(d2) : 0.0;
    }
    dd[ia][ib] = d;
  }
  __syncthreads();
  if (e < 32) {
    double sum = 0.0;
    for (int j = 0; j < 16; ++j) sum += e < 16 ? dd[e][j] : dd[j][e - 16];
    store_wt(rsum + p * 32 + e, sum);
  }
  if (!last_arrival(ticket, unsigned(gridDim.x), &flag)) return;
  const int a = e;
  double sum = 0.0;
  if (a < n && a < 256) {
    const int ta = a >> 4, i = a & 15;
    for (int v = 0; v < T; ++v)
      sum += ta <= v ? rsum[pair_index(ta, v, T) * 32 + i]
                     : rsum[pair_index(v, ta, T) * 32 + 16 + i];
  }
  if (a < 256) tot[a] = sum;
  __syncthreads();
  if (a == 0) {
    int best = 0;
    for (int b = 1; b < n; ++b)
      if (tot[b] < tot[best]) best = b;
    *centre = best;
  }
}

// gram_key_kernel (grid nseg x ntpg: the pair's Gram block summed over the
// key's first-level groups, d² and bound at (a, b) and (b, a)) with the
// finish fused: the last of tile pair p's nseg workgroups finishes the
// block's pairs (finish_pair_sym, as gram_finish_kernel) from every key's
// d² and bound.  The first-level sums stay a kernel of their own
// (gram_reduce1_kernel, one workgroup per group and tile pair): summed here
// per key they ran one memory round trip per group, and the largest key's
// ~20 groups in a row took 90 µs at C4 (profiles/r06/gram_fused_ab*.jsonl).
__global__ __launch_bounds__(320) void gram_keyfin_kernel(
    const double *__restrict__ red, GramCtl ctl, int n, int T,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, double *__restrict__ segsq, double *__restrict__ err,
    unsigned *__restrict__ ticket, double tol, float *__restrict__ D,
    uint32_t *__restrict__ ill, float *__restrict__ B,
    double *__restrict__ D64) {
  __shared__ double dg[32];
  __shared__ int flag;
  const int s = blockIdx.x, p = blockIdx.y, e = threadIdx.x;
  const int ntpg = T * (T + 1) / 2;
  int t, u;
  tp_tiles(p, T, t, u);
  // waves 0-3 the block's 256 entries, wave 4 the two tiles' diagonals
  // (at the same time: the first build summed them behind the entries)
  double gab = 0.0;
  if (e < 256) {
    gab = sum_items(red, ctl.gprefix[s], ctl.gprefix[s + 1], ntpg, p, e);
  } else if (e < 256 + 32) {
    const int d = e - 256;
    const int tt = d < 16 ? t : u;
    dg[d] = sum_items(red, ctl.gprefix[s], ctl.gprefix[s + 1], ntpg,
                      pair_index(tt, tt, T), diag_entry(d & 15));
  }
  __syncthreads();
  const int l = e & 63, r = (e >> 6) & 3, ia = 4 * (l >> 4) + r, ib = l & 15;
  const int a = e < 256 ? 16 * t + ia : n, b = 16 * u + ib;
  if (a < n && b < n && !(t == u && ia > ib)) {
    double d2, er;
    segsq_pair(dg[ia], dg[16 + ib], gab, a == b, seg_end[s] - seg_lo[s], d2,
               er);
    const int64_t o = int64_t(s) * n * n;
    store_wt(segsq + o + int64_t(a) * n + b, d2);
    store_wt(err + o + int64_t(a) * n + b, er);
    store_wt(segsq + o + int64_t(b) * n + a, d2);
    store_wt(err + o + int64_t(b) * n + a, er);
  }
  if (!D) return;
  if (!last_arrival(ticket + p, unsigned(nseg), &flag)) return;
  if (a < n && b < n)
    finish_pair_sym(a * n + b, b * n + a, segsq, err, n, nseg, tol, D, ill,
                    B, D64);
}

// The finish of a sharded call, after the ranks' d² and bounds were summed
// (fsagg_pairgram_finish_f32): finish_pair on every pair.
__global__ __launch_bounds__(256) void gram_finish_kernel(
    const double *__restrict__ segsq, const double *__restrict__ err, int n,
    int nseg, double tol, float *__restrict__ D, uint32_t *__restrict__ ill,
    float *__restrict__ B, double *__restrict__ D64) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q < n * n) finish_pair(q, segsq, err, n, nseg, tol, D, ill, B, D64);
}

// n > 64 (T > 4 tiles): 8-tile workgroups.  The plane-line form above
// stages and splits every tile on 4 lines (13 workgroups per chunk at
// T = 13) and each wave forms every pair of its line for a quarter of the
// k-steps, so each split serves 10 pairs but every tile is split 4 times
// over.  Here a workgroup of 8 waves holds 8 tiles: per stage (64
// coordinates = 2 k-steps) wave w splits ITS tile's limbs once into LDS and
// then forms its share of the workgroup's tile pairs from there — every pair
// owned by one wave for all k-steps, so no cross-wave sum — reading its own
// tile's fragments once per k-step and each partner's per pair.  T <= 8
// (n <= 128): one workgroup per chunk holds every tile.  9 <= T <= 13: four
// workgroups per chunk, tile sets {0-7}, {5-12}, {0-4, 8-10}, {0-4, 11, 12},
// each forming only the pairs no earlier set holds (36 + 30 + 15 + 10 = 91
// pairs, each exactly once; 32 tile splits per chunk against 52 on lines).
// LDS: the raw stage (128 rows × 256 B, global_load_lds with the source
// swizzle of kGramStaged) and the limbs of two k-steps (2 × 8 tiles × 3 ×
// 1 KiB) = 80 KiB, two workgroups per CU; the centre's values come from
// global memory one stage ahead (every workgroup of a chunk reads the same
// row, from L2).
constexpr int kB8Waves = 8;
constexpr int kB8Stage = 2 * kKStep;                // 64 coordinates
constexpr int kB8RowBytes = kB8Stage * 4;           // 256 B
// Two configurations: 8 tiles on 8 waves (types 0-4 below: T <= 8, or the
// four-workgroup covering of T <= 13 under the A/B setting), and all 13
// tiles on 16 waves (type 5: 9 <= T <= 13, one workgroup per chunk).
template <int NT, int W>
struct B8Cfg {
  static constexpr int kBlk = W * kWave;
  static constexpr int kRaw = 16 * NT * kB8RowBytes;   // 32 / 52 KiB
  static constexpr int kLimbs = 2 * NT * 3 * 1024;     // 48 / 78 KiB
  static constexpr int kPieces = 4 * NT;               // 4-row pieces
  static constexpr int kMy = (kPieces + W - 1) / W;    // per wave
  static constexpr int kMaxPairs = NT == 8 ? 5 : 6;
};
// global tile of local tile lt, per block type (0: the one block of T <= 8;
// 1-4: the four blocks of 9 <= T <= 13; 5-10: the six blocks of
// 14 <= T <= 16 — the tile groups A = 0-3, B = 4-7, C = 8-11, D = 12-15 as
// A∪B and C∪D, every pair inside each, then A∪C, A∪D, B∪C, B∪D, the
// cross pairs only: 36 + 36 + 4 · 16 = 136 pairs, each once); -1 = none
__constant__ int8_t kB8Tiles[11][8] = {
    {0, 1, 2, 3, 4, 5, 6, 7},   {0, 1, 2, 3, 4, 5, 6, 7},
    {5, 6, 7, 8, 9, 10, 11, 12}, {0, 1, 2, 3, 4, 8, 9, 10},
    {0, 1, 2, 3, 4, 11, 12, -1},
    {0, 1, 2, 3, 4, 5, 6, 7},     {8, 9, 10, 11, 12, 13, 14, 15},
    {0, 1, 2, 3, 8, 9, 10, 11},   {0, 1, 2, 3, 12, 13, 14, 15},
    {4, 5, 6, 7, 8, 9, 10, 11},   {4, 5, 6, 7, 12, 13, 14, 15}};
// wave w's local tile pairs lo·8 + hi (lo <= hi), -1 none; types 0, 1, 5
// and 6: every pair of 8 tiles, (w, w + d mod 8) for d <= 3 and (w, w + 4)
// for w < 4; type 2: without the pairs inside tiles 0-2 (block 1 holds
// them); types 3, 4: tiles 0-4 against 5-7 / 5-6; types 7-10: local tiles
// 0-3 against 4-7, wave w the pairs of tile w & 3 with 4 + 2(w >> 2) and
// the next (one first operand per wave)
__constant__ int8_t kB8Pairs[11][8][5] = {
    {{0, 1, 2, 3, 4}, {9, 10, 11, 12, 13}, {18, 19, 20, 21, 22},
     {27, 28, 29, 30, 31}, {36, 37, 38, 39, -1}, {45, 46, 47, 5, -1},
     {54, 55, 6, 14, -1}, {63, 7, 15, 23, -1}},
    {{0, 1, 2, 3, 4}, {9, 10, 11, 12, 13}, {18, 19, 20, 21, 22},
     {27, 28, 29, 30, 31}, {36, 37, 38, 39, -1}, {45, 46, 47, 5, -1},
     {54, 55, 6, 14, -1}, {63, 7, 15, 23, -1}},
    {{3, 4, -1, -1, -1}, {11, 12, 13, -1, -1}, {19, 20, 21, 22, -1},
     {27, 28, 29, 30, 31}, {36, 37, 38, 39, -1}, {45, 46, 47, 5, -1},
     {54, 55, 6, 14, -1}, {63, 7, 15, 23, -1}},
    {{5, 6, 7, -1, -1}, {13, 14, 15, -1, -1}, {21, 22, 23, -1, -1},
     {29, 30, 31, -1, -1}, {37, 38, 39, -1, -1}, {-1, -1, -1, -1, -1},
     {-1, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}},
    {{5, 6, -1, -1, -1}, {13, 14, -1, -1, -1}, {21, 22, -1, -1, -1},
     {29, 30, -1, -1, -1}, {37, 38, -1, -1, -1}, {-1, -1, -1, -1, -1},
     {-1, -1, -1, -1, -1}, {-1, -1, -1, -1, -1}},
#define FSAGG_B8_ALL                                                       \
  {{0, 1, 2, 3, 4}, {9, 10, 11, 12, 13}, {18, 19, 20, 21, 22},              \
   {27, 28, 29, 30, 31}, {36, 37, 38, 39, -1}, {45, 46, 47, 5, -1},         \
   {54, 55, 6, 14, -1}, {63, 7, 15, 23, -1}}
#define FSAGG_B8_CROSS                                                     \
  {{4, 5, -1, -1, -1}, {12, 13, -1, -1, -1}, {20, 21, -1, -1, -1},          \
   {28, 29, -1, -1, -1}, {6, 7, -1, -1, -1}, {14, 15, -1, -1, -1},          \
   {22, 23, -1, -1, -1}, {30, 31, -1, -1, -1}}
    FSAGG_B8_ALL, FSAGG_B8_ALL, FSAGG_B8_CROSS, FSAGG_B8_CROSS,
    FSAGG_B8_CROSS, FSAGG_B8_CROSS};
#undef FSAGG_B8_ALL
#undef FSAGG_B8_CROSS
// 13 tiles on 16 waves: wave w's pairs t·16 + u (t <= u), -1 none — wave
// w < 13 its own tile against (w + d mod 13), d = 0 … 5; the seventh of
// each (d = 6) and the rest spread over waves 13-15 (91 pairs, <= 6 each)
__constant__ uint8_t kWidePairs[16][6] = {
    {0, 1, 2, 3, 4, 5},          {17, 18, 19, 20, 21, 22},
    {34, 35, 36, 37, 38, 39},    {51, 52, 53, 54, 55, 56},
    {68, 69, 70, 71, 72, 73},    {85, 86, 87, 88, 89, 90},
    {102, 103, 104, 105, 106, 107}, {119, 120, 121, 122, 123, 124},
    {136, 137, 138, 139, 140, 8}, {153, 154, 155, 156, 9, 25},
    {170, 171, 172, 10, 26, 42}, {187, 188, 11, 27, 43, 59},
    {204, 12, 28, 44, 60, 76},   {6, 23, 40, 57, 74, 91},
    {7, 24, 41, 58, 75, 108},    {92, 255, 255, 255, 255, 255}};

// the 8 values of lane (row rr, group g) for k-step ks of a raw stage
__device__ __forceinline__ void b8_read8(const char *buf, int rr, int ks,
                                         int g, float (&v)[8]) {
  typedef __attribute__((address_space(3))) const f32x4 lds_f32x4;
  const int c0 = 8 * ks + g, c1 = c0 + 4;
  const char *r = buf + rr * kB8RowBytes;
  const f32x4 x = *(lds_f32x4 *)(uintptr_t)(r + 16 * (c0 ^ (rr & 15)));
  const f32x4 y = *(lds_f32x4 *)(uintptr_t)(r + 16 * (c1 ^ (rr & 15)));
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
}

struct Limbs3 {
  frag8 h, m, l;
};

// limb fragments (k-step ks, local tile t) of this lane: [ks][t][h|m|l]
template <int NT>
__device__ __forceinline__ frag8 *b8_limb(char *limbs, int ks, int t, int lb,
                                         int lane) {
  return reinterpret_cast<frag8 *>(limbs + ((ks * NT + t) * 3 + lb) * 1024 +
                                   lane * 16);
}

template <int NT>
__device__ __forceinline__ Limbs3 b8_load(char *limbs, int ks, int t,
                                          int lane) {
  Limbs3 f;
  f.h = *b8_limb<NT>(limbs, ks, t, 0, lane);
  f.m = *b8_limb<NT>(limbs, ks, t, 1, lane);
  f.l = *b8_limb<NT>(limbs, ks, t, 2, lane);
  return f;
}

// the six limb products of (a, b) for one k-step, small first (as
// kstep_mfma), into fp64
__device__ __forceinline__ void b8_pair(const Limbs3 &a, const Limbs3 &b,
                                        double (&acc)[4]) {
  f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, x, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] += double(x[r]);
}

// NT tiles on W waves (B8Cfg): per stage (64 coordinates = 2 k-steps) wave
// w < NT splits local tile w's limbs into LDS once, then every wave forms
// its pairs (t, u) from there — each pair owned by one wave for all
// k-steps, so no cross-wave sum; the first operand's fragments are kept
// while consecutive pairs share it.  NT = 8: block type 0-4 (kB8Tiles /
// kB8Pairs); NT = 13: one workgroup with every tile (kWidePairs).
template <int NT, int W, bool CENTRED>
__global__ __launch_bounds__(W * kWave)
__attribute__((amdgpu_waves_per_eu(4))) void gram_block8_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n, int T, int NB,
    const int64_t *__restrict__ seg_lo, const int64_t *__restrict__ seg_end,
    int nseg, GramCtl ctl, int64_t w, int64_t cap,
    const int *__restrict__ centre, double *__restrict__ partial) {
  typedef B8Cfg<NT, W> C;
  __shared__ __attribute__((aligned(1024))) char raw[C::kRaw];
  __shared__ __attribute__((aligned(1024))) char limbs[C::kLimbs];
  const int *__restrict__ prefix = ctl.prefix;
  // blocks b and b + 8 share an XCD: a chunk's NB workgroups run on one
  // XCD together and read its rows from that L2 after the first
  const int kq = int(blockIdx.x >> 3);
  const int chunk = (kq / NB) * 8 + int(blockIdx.x & 7);
  const int type = NB == 1 ? 0 : (NB == 6 ? 5 : 1) + kq % NB;
  if (chunk >= prefix[nseg]) return;  // whole workgroup
  int s = 0;
  while (prefix[s + 1] <= chunk) ++s;
  const int q = chunk - prefix[s];
  const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);
  const int lane = int(threadIdx.x) % kWave, g = lane >> 4;
  int64_t send = seg_end[s];
  if (cap > 0 && send > seg_lo[s] + cap) send = seg_lo[s] + cap;
  const int64_t c0 = seg_lo[s] + int64_t(q) * w;
  const int64_t c1 = min(c0 + w, send);
  const int64_t len = c1 > c0 ? c1 - c0 : 0;
  const float *const *rows = tab + int64_t(s) * ss;
  auto gtile = [&](int lt) {
    return NT == 8 ? int(kB8Tiles[type][lt]) : lt;
  };
  auto client = [&](int lt, int r) {  // row r of local tile lt, clamped
    const int gt = gtile(lt);
    const int j = 16 * gt + r;
    return gt < 0 || j >= n ? n - 1 : j;
  };
  // this wave's own tile row (the split) and the centre row
  const bool splits = wv < NT;
  const float *own = rows[client(splits ? wv : 0, lane & 15)];
  const float *crow = CENTRED ? rows[*centre] : nullptr;
  // the raw stage: pieces k = wv + W·m, lane l → row 4k + (l >> 4), 16-B
  // chunk l & 15, stored at slot (l & 15) ^ (row & 15) of that row
  const float *src[C::kMy];
  uint32_t dst[C::kMy];
  bool ok = true;
#pragma unroll
  for (int m = 0; m < C::kMy; ++m) {
    const int k = wv + W * m;
    const int rr = 4 * (k < C::kPieces ? k : 0) + (lane >> 4);
    const float *rp = rows[client(rr >> 4, rr & 15)];
    ok = ok && al16(rp + c0);
    src[m] = rp + c0 + 4 * (lane & 15);
    dst[m] = uint32_t(rr * kB8RowBytes + 16 * ((lane & 15) ^ (rr & 15)));
  }
  if (CENTRED) ok = ok && al16(crow + c0);
  // the workgroup's agreement through the (still unused) limb area: a
  // __syncthreads_and would take LDS of its own past the 80 KiB that lets
  // two 8-wave workgroups share a CU
  uint32_t *flag = reinterpret_cast<uint32_t *>(limbs);
  if (lane == 0) flag[wv] = __all(ok) ? 1u : 0u;
  __syncthreads();
  bool vec = true;
#pragma unroll
  for (int v = 0; v < W; ++v) vec = vec && flag[v] != 0u;
  __syncthreads();  // read before any limb is written

  // this wave's pairs (wave-uniform): local (t, u), t <= u
  int np = 0;
  int pt[C::kMaxPairs], pu[C::kMaxPairs];
#pragma unroll
  for (int p = 0; p < C::kMaxPairs; ++p) {
    int e, t, u;
    if constexpr (NT == 8) {
      e = kB8Pairs[type][wv][p];
      t = e >= 0 ? e >> 3 : 0;
      u = e >= 0 ? e & 7 : 0;
    } else {
      e = kWidePairs[wv][p] == 255 ? -1 : int(kWidePairs[wv][p]);
      t = e >= 0 ? e >> 4 : 0;
      u = e >= 0 ? e & 15 : 0;
    }
    pt[p] = __builtin_amdgcn_readfirstlane(t);
    pu[p] = __builtin_amdgcn_readfirstlane(u);
    np += e >= 0 ? 1 : 0;
  }
  np = __builtin_amdgcn_readfirstlane(np);
  double acc[C::kMaxPairs][4];
#pragma unroll
  for (int p = 0; p < C::kMaxPairs; ++p)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[p][r] = 0.0;

  const Neg kn = neg_consts();
  // the products of k-step ks from the limbs (measured and not kept: the
  // pairs' chains interleaved in a branch-free body — at the 128-VGPR
  // budget it spills, at one 8-wave workgroup per CU n = 100 took 1.39 ms
  // against 0.93)
  auto mfma_phase = [&](int ks) {
    Limbs3 a;
    int at = -1;
#pragma unroll
    for (int p = 0; p < C::kMaxPairs; ++p) {
      if (p < np) {
        if (pt[p] != at) {
          a = b8_load<NT>(limbs, ks, pt[p], lane);
          at = pt[p];
        }
        if (pu[p] == pt[p]) {
          b8_pair(a, a, acc[p]);
        } else {
          const Limbs3 b = b8_load<NT>(limbs, ks, pu[p], lane);
          b8_pair(a, b, acc[p]);
        }
      }
    }
  };
  auto split_to = [&](int ks, const float (&x)[8]) {
    frag8 h, m, l;
    split3(x, kn, h, m, l);
    *b8_limb<NT>(limbs, ks, wv, 0, lane) = h;
    *b8_limb<NT>(limbs, ks, wv, 1, lane) = m;
    *b8_limb<NT>(limbs, ks, wv, 2, lane) = l;
  };

  const int nstage = vec ? int(len / kB8Stage) : 0;
  float cb[2][8];
  auto centre_load = [&](int st) {
    if (CENTRED) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        ld8(crow + c0 + int64_t(st) * kB8Stage + ks * kKStep + 4 * g, cb[ks]);
    }
  };
  // a stage's rows in flight in registers (16-B loads, each row's 256 B
  // by one 16-lane group), written to the raw stage once every wave has
  // read the previous one: the loads of stage st + 2 fly while stage st's
  // products are formed and stage st + 1 is split
  f32x4 pre[C::kMy];
  auto fetch = [&](int st) {
#pragma unroll
    for (int m = 0; m < C::kMy; ++m)
      if (wv + W * m < C::kPieces)
        pre[m] = gld_nt(reinterpret_cast<const f32x4 *>(
            src[m] + int64_t(st) * kB8Stage));
  };
  auto put = [&]() {
    typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
#pragma unroll
    for (int m = 0; m < C::kMy; ++m)
      if (wv + W * m < C::kPieces)
        *(lds_f32x4 *)(uintptr_t)(raw + dst[m]) = pre[m];
  };
  if (nstage > 0) {
    fetch(0);
    centre_load(0);
    put();
    if (nstage > 1) fetch(1);
  }
  for (int st = 0; st < nstage; ++st) {
    // stage st is in the raw buffer (every wave's part), and every wave is
    // done reading the limbs of stage st − 1
    __syncthreads();
    if (splits) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float x[8];
        b8_read8(raw, 16 * wv + (lane & 15), ks, g, x);
        if (CENTRED) {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] -= cb[ks][j];
        }
        split_to(ks, x);
      }
    }
    // the limbs are written and the raw stage read by every wave
    __syncthreads();
    if (st + 1 < nstage) {
      put();
      centre_load(st + 1);
      if (st + 2 < nstage) fetch(st + 2);
    }
    mfma_phase(0);
    mfma_phase(1);
  }
  // the rest (unaligned rows: everything; aligned: the last partial stage),
  // one k-step at a time from global memory
  const int nall = int((len + kKStep - 1) / kKStep);
  for (int i = 2 * nstage; i < nall; ++i) {
    const int64_t k0 = c0 + int64_t(i) * kKStep;
    __syncthreads();  // every wave is done with the limbs
    if (splits) {
      float x[8], cc[8];
      ld8_tail(own, k0, c1, g, x);
      if (CENTRED) {
        ld8_tail(crow, k0, c1, g, cc);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] -= cc[j];
      }
      split_to(0, x);
    }
    __syncthreads();
    mfma_phase(0);
  }
  const int ntpg = T * (T + 1) / 2;
  double *out = partial + int64_t(chunk) * ntpg * 256;
#pragma unroll
  for (int p = 0; p < C::kMaxPairs; ++p) {
    if (p >= np) continue;
    const int a = gtile(pt[p]), b = gtile(pu[p]);
    if (a < 0 || b < 0 || b >= T) continue;  // absent tiles
    double *o = out + int64_t(pair_index(a, b, T)) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r * 64 + lane] = acc[p][r];
  }
}

// n > 64: 1 (default) = up to 7 tiles (n <= 112) the n <= 64 kernel's
// form — one 4-wave workgroup per chunk holding every tile, one per CU —
// then gram_block8_kernel's 8 tiles, all 13 on 16 waves above; 2 = 8-tile
// workgroups for every n > 64 (four per chunk above 128); 3 = the one-
// workgroup form for every T <= 8, 13 tiles above as 1; 0 = plane lines
// throughout (fsagg_pairgram_set_block8, A/B)
std::atomic<int> g_block8{1};
// 1 (default): compact stage buffers (the n client rows), three of them
// where they fit (two stages in flight); 0: the round-5 full-tile stages
// (16·NT rows + the centre's, one in flight) — fsagg_pairgram_set_stages,
// A/B
std::atomic<int> g_compact{1};
// main-pass chunks (n <= 112 forms): about kMainChunks workgroups — two
// rounds at two per CU; fsagg_pairgram_set_chunks, A/B
std::atomic<int> g_main_chunks{kMainChunks};
// A/B: bits 0-1 pick the main-pass workgroups that start late (1: odd
// blocks, 2: bit 8, 3: bit 9), bits 2+ the delay in 512-cycle sleeps;
// fsagg_pairgram_set_desync
std::atomic<int> g_desync{0};
// 1 (default): the fused tail — the centre picked by the last pair-sum
// workgroup, key + finish in gram_keyfin_kernel (six launches per chain);
// 0: the round-5 eight launches (fsagg_pairgram_set_fused, A/B; the results
// are bit-identical)
std::atomic<int> g_fused{1};

struct GramPlan {
  int nt;              // tiles of 16 clients
  bool lines;          // nt > kFullTiles: several workgroups per chunk
  bool block8;         // ... 8-tile workgroups (else plane lines)
  bool wide;           // ... one 13-tile workgroup of 16 waves
  int nlines;          // workgroups per chunk: 13 / 7 lines, or 1 / 4 blocks
  int ntpg;            // tile pairs
  int64_t w;           // main chunk length (multiple of kUnit)
  int main_chunks;     // upper bounds
  int sample_chunks;
  int main_groups;
};

GramPlan gram_plan(int n, int64_t numel, int nseg) {
  GramPlan pl;
  pl.nt = (n + 15) / 16;
  pl.lines = pl.nt > kFullTiles;
  // tile-split workgroups where they measured faster than the plane lines
  // (profiles/r05/gram_block8_ab.jsonl): one 8-tile workgroup per chunk
  // for T <= 8 (n = 100: 0.91 against 1.09 ms, n = 128: 0.99 against
  // 2.91), one 13-tile workgroup of 16 waves for 9 <= T <= 13 (n = 200:
  // 2.57 against 3.21 ms); the four 8-tile workgroups of the A/B setting 2
  // measured slower (3.8 ms at n = 200)
  const int b8 = g_block8.load(std::memory_order_relaxed);
  // T > 13: the six 8-tile workgroups whatever the setting (the plane lines
  // and the 13-tile workgroup stop at 13)
  pl.block8 = pl.lines && (b8 != 0 || pl.nt > kPlaneTiles);
  // 9 <= T <= 13: one 16-wave workgroup with all 13 tiles (setting 1), or
  // the four 8-tile workgroups (setting 2)
  pl.wide = pl.block8 && pl.nt > kB8Waves && pl.nt <= kPlaneTiles &&
            (b8 == 1 || b8 == 3);
  // up to kOneMaxTiles (setting 3: 8) tiles the n <= 64 kernel's form: one
  // 4-wave workgroup per chunk, each wave splitting every tile of its own
  // k-steps and forming every pair from registers (up to 256 VGPRs + AGPRs,
  // one workgroup per CU) — profiles/r05/gram_full_ab.jsonl: n = 66 0.49
  // against 0.70 ms, n = 90 0.66 / 0.84, n = 100 0.90 / 0.97, but n = 113
  // 1.12 / 1.01 and n = 128 1.13 / 1.03 against the 8-tile workgroup
  if (pl.lines && (b8 == 1 || b8 == 3) &&
      pl.nt <= (b8 == 3 ? kB8Waves : kOneMaxTiles))
    pl.lines = pl.block8 = pl.wide = false;
  pl.nlines = !pl.lines ? 1
              : pl.block8 ? (pl.nt <= kB8Waves || pl.wide
                                 ? 1
                                 : (pl.nt <= kPlaneTiles ? 4 : 6))
                          : (pl.nt <= 7 ? 7 : 13);
  pl.ntpg = ntp_of(pl.nt);
  // ~kMainChunks workgroups; LINES: ~kLineBlocks over all the lines
  // (fewer, longer chunks: less partial traffic); 8-tile blocks: ~2048
  // workgroups of 512 threads (1024 chunks of one block, 512 of four)
  const int64_t target =
      !pl.lines ? int64_t(g_main_chunks.load(std::memory_order_relaxed))
      : pl.block8 ? (pl.nlines == 1 ? 1024 : 512)
                  : (kLineBlocks / pl.nlines > 64 ? kLineBlocks / pl.nlines
                                                  : 64);
  int64_t w = (numel + target - 1) / target;
  w = (w + kUnit - 1) / kUnit * kUnit;
  if (w < kUnit) w = kUnit;
  if (w > kMaxW) w = kMaxW;
  pl.w = w;
  pl.main_chunks = int(numel / w) + nseg + 1;
  pl.main_groups = pl.main_chunks / kRed + nseg + 1;
  const int per_key = int((kSampleCoords + kSampleChunk - 1) / kSampleChunk);
  pl.sample_chunks = nseg * per_key;
  return pl;
}

// chunk-kernel grid: one workgroup per chunk, or per chunk and plane line
// with the chunks rounded up to the 8 XCDs (LINES)
unsigned chunk_grid(const GramPlan &pl, int chunks) {
  return pl.lines ? unsigned((chunks + 7) / 8 * 8 * pl.nlines)
                  : unsigned(chunks);
}

struct GramWs {
  GramCtl cs, cm;          // sample and main pass plans
  int *centre;
  unsigned *tickets;       // [ntpg] keyfin, [ntpg] the centre pick
  double *partial, *red, *rsum;
};

size_t gram_ws_layout(int n, int64_t numel, int nseg, void *ws, GramWs *w) {
  const GramPlan pl = gram_plan(n, numel, nseg);
  const size_t ntp = size_t(pl.ntpg);
  const size_t chunks = size_t(pl.main_chunks > pl.sample_chunks
                                   ? pl.main_chunks
                                   : pl.sample_chunks);
  const size_t groups = size_t(pl.main_groups);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += align256(bytes);
    return static_cast<char *>(ws) + o;
  };
  auto ctl = [&]() {
    int *p = reinterpret_cast<int *>(take(sizeof(int) * 2 * size_t(nseg + 1)));
    GramCtl c;
    c.prefix = p;
    c.gprefix = p + (nseg + 1);
    c.desync = g_desync.load(std::memory_order_relaxed);
    return c;
  };
  const GramCtl cs = ctl(), cm = ctl();
  char *p_c = take(256),
       *p_tk = take(sizeof(unsigned) * (ntp + 1)),
       *p_rs = take(sizeof(double) * ntp * 32),
       *p_red = take(sizeof(double) * groups * ntp * 256),
       *p_part = take(sizeof(double) * chunks * ntp * 256);
  if (w) {
    w->cs = cs;
    w->cm = cm;
    w->centre = reinterpret_cast<int *>(p_c);
    w->tickets = reinterpret_cast<unsigned *>(p_tk);
    w->rsum = reinterpret_cast<double *>(p_rs);
    w->red = reinterpret_cast<double *>(p_red);
    w->partial = reinterpret_cast<double *>(p_part);
  }
  return off;
}

// Seven launches (eight with the finish): both plans; the sample pass, the
// tile pairs' distance sums and the centre; the centred main pass, its group
// sums, and per key and tile pair the Gram block, d² and bounds.
// the sample (CENTRED false) or main pass's chunk kernel
template <int NT, bool LINES, bool CENTRED>
void gram_pass(const float *const *tab, int64_t ss, int n,
               const int64_t *seg_lo, const int64_t *seg_end, int nseg,
               const GramPlan &pl, GramCtl ctl, int64_t w, int64_t cap,
               const int *centre, double *partial, int chunks,
               hipStream_t st) {
  if constexpr (LINES) {
    if (pl.wide)
      hipLaunchKernelGGL((gram_block8_kernel<13, 16, CENTRED>),
                         dim3(chunk_grid(pl, chunks)), dim3(16 * kWave), 0,
                         st, tab, ss, n, pl.nt, pl.nlines, seg_lo, seg_end,
                         nseg, ctl, w, cap, centre, partial);
    else if (pl.block8)
      hipLaunchKernelGGL((gram_block8_kernel<8, kB8Waves, CENTRED>),
                         dim3(chunk_grid(pl, chunks)), dim3(kB8Waves * kWave),
                         0, st, tab, ss, n, pl.nt, pl.nlines, seg_lo, seg_end,
                         nseg, ctl, w, cap, centre, partial);
    else  // plane lines re-read tiles through L2: plain loads
      hipLaunchKernelGGL((gram_chunk_kernel<NT, CENTRED, true, 0, 2, false,
                                            false, 0>),
                         dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab,
                         ss, n, pl.nt, seg_lo, seg_end, nseg, ctl, w, cap,
                         centre, partial);
  } else if constexpr (NT > kFullTiles) {
    // NT > 4 (one workgroup per CU, up to 256 VGPRs + AGPRs): the full-tile
    // stages — the compact form spilled there (n = 100: 0.99 against
    // 0.89 ms, profiles/r06/gram_stages_ab.jsonl); stages 4: plain loads
    if (g_compact.load(std::memory_order_relaxed) == 4)
      hipLaunchKernelGGL((gram_chunk_kernel<NT, CENTRED, false, 0, 2, false,
                                            false, 0>),
                         dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab,
                         ss, n, pl.nt, seg_lo, seg_end, nseg, ctl, w, cap,
                         centre, partial);
    else
      hipLaunchKernelGGL((gram_chunk_kernel<NT, CENTRED, false>),
                         dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab,
                         ss, n, pl.nt, seg_lo, seg_end, nseg, ctl, w, cap,
                         centre, partial);
  } else if (g_compact.load(std::memory_order_relaxed) == 0) {
    // A/B: the round-5 full-tile stages (16·NT rows + the centre), one in
    // flight
    hipLaunchKernelGGL((gram_chunk_kernel<NT, CENTRED, false>),
                       dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab,
                       ss, n, pl.nt, seg_lo, seg_end, nseg, ctl, w, cap,
                       centre, partial);
  } else if (g_compact.load(std::memory_order_relaxed) == 3) {
    // A/B: the compact stages with the MFMA cluster at priority 1
    if ((n + 1) / 2 <= compact_maxi3<NT>())
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, compact_maxi3<NT>(), 3,
                             false, true>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
    else
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, 8 * NT, 2, false, true>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
  } else if (g_compact.load(std::memory_order_relaxed) == 4) {
    // A/B: the default compact stages with plain (temporal) loads
    if ((n + 1) / 2 <= compact_maxi3<NT>())
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, compact_maxi3<NT>(), 3,
                             false, false, 0>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
    else
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, 8 * NT, 2, false, false, 0>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
  } else if (g_compact.load(std::memory_order_relaxed) == 2) {
    // early release: every buffer's stage in flight under the compute
    if ((n + 1) / 2 <= compact_maxi3<NT>())
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, compact_maxi3<NT>(), 3,
                             true>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
    else
      hipLaunchKernelGGL(
          (gram_chunk_kernel<NT, CENTRED, false, 8 * NT, 2, true>),
          dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
          seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
  } else if ((n + 1) / 2 <= compact_maxi3<NT>()) {
    // three compact stage buffers: two stages in flight
    hipLaunchKernelGGL(
        (gram_chunk_kernel<NT, CENTRED, false, compact_maxi3<NT>(), 3>),
        dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab, ss, n, pl.nt,
        seg_lo, seg_end, nseg, ctl, w, cap, centre, partial);
  } else {
    hipLaunchKernelGGL((gram_chunk_kernel<NT, CENTRED, false, 8 * NT, 2>),
                       dim3(chunk_grid(pl, chunks)), dim3(kBlk), 0, st, tab,
                       ss, n, pl.nt, seg_lo, seg_end, nseg, ctl, w, cap,
                       centre, partial);
  }
}

template <int NT, bool LINES>
void gram_launch(const float *const *tab, int64_t ss, int n,
                 const int64_t *seg_lo, const int64_t *seg_end, int nseg,
                 const GramPlan &pl, const GramWs &w, double *segsq,
                 double *err, double tol, float *D, uint32_t *ill, float *B,
                 double *D64, hipStream_t st) {
  const int T = pl.nt;
  const bool fused = g_fused.load(std::memory_order_relaxed) != 0;
  hipLaunchKernelGGL(gram_prefix_kernel, dim3(1), dim3(2 * kWave), 0, st,
                     seg_lo, seg_end, nseg, kSampleChunk, kSampleCoords, pl.w,
                     w.cs, w.cm, w.tickets, pl.ntpg + 1);
  // 1. the centre: Gram of the first kSampleCoords of every key, raw
  gram_pass<NT, LINES, false>(tab, ss, n, seg_lo, seg_end, nseg, pl, w.cs,
                              kSampleChunk, kSampleCoords, nullptr, w.partial,
                              pl.sample_chunks, st);
  if (fused) {
    hipLaunchKernelGGL(gram_centre_fused_kernel, dim3(unsigned(pl.ntpg)),
                       dim3(320), 0, st, w.partial, w.cs, nseg, n, T, w.rsum,
                       w.tickets + pl.ntpg, w.centre);
  } else {
    hipLaunchKernelGGL(gram_centre_pairs_kernel, dim3(unsigned(pl.ntpg)),
                       dim3(256), 0, st, w.partial, w.cs, nseg, n, T, w.rsum);
    hipLaunchKernelGGL(gram_centre_pick_kernel, dim3(1), dim3(256), 0, st,
                       w.rsum, n, T, w.centre);
  }
  // 2. the centred Gram of every key, its d² and bounds
  gram_pass<NT, LINES, true>(tab, ss, n, seg_lo, seg_end, nseg, pl, w.cm,
                             pl.w, int64_t(0), w.centre, w.partial,
                             pl.main_chunks, st);
  hipLaunchKernelGGL(gram_reduce1_kernel,
                     dim3(unsigned(pl.main_groups), unsigned(pl.ntpg)),
                     dim3(256), 0, st, w.partial, w.cm, nseg, pl.ntpg, w.red);
  if (fused) {
    hipLaunchKernelGGL(gram_keyfin_kernel,
                       dim3(unsigned(nseg), unsigned(pl.ntpg)), dim3(320), 0,
                       st, w.red, w.cm, n, T, seg_lo, seg_end, nseg, segsq,
                       err, w.tickets, tol, D, ill, B, D64);
    return;
  }
  hipLaunchKernelGGL(gram_key_kernel,
                     dim3(unsigned(nseg), unsigned(pl.ntpg)), dim3(256), 0,
                     st, w.red, w.cm, n, T, seg_lo, seg_end, segsq, err);
  if (D)
    hipLaunchKernelGGL(gram_finish_kernel,
                       dim3(unsigned((int64_t(n) * n + 255) / 256)),
                       dim3(256), 0, st, segsq, err, n, nseg, tol, D, ill,
                       B, D64);
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_pairgram_set_block8(int on) {
  return g_block8.exchange(on < 0 ? 1 : (on > 3 ? 3 : on));
}

extern "C" int fsagg_pairgram_set_fused(int on) {
  return g_fused.exchange(on < 0 ? 1 : (on > 0 ? 1 : 0));
}

extern "C" int fsagg_pairgram_set_stages(int mode) {
  return g_compact.exchange(mode < 0 ? 1 : (mode > 4 ? 4 : mode));
}

extern "C" int fsagg_pairgram_set_desync(int mode) {
  return g_desync.exchange(mode < 0 ? 0 : mode);
}

extern "C" int fsagg_pairgram_set_chunks(int chunks) {
  return g_main_chunks.exchange(chunks <= 0 ? kMainChunks
                                            : (chunks < 64 ? 64 : chunks));
}

extern "C" int64_t fsagg_pairgram_knobs(void) {
  return int64_t(g_block8.load(std::memory_order_relaxed) & 3) |
         (int64_t(g_compact.load(std::memory_order_relaxed) & 7) << 2) |
         (int64_t(g_fused.load(std::memory_order_relaxed) & 1) << 5) |
         (int64_t(g_desync.load(std::memory_order_relaxed) & 0xffff) << 6) |
         (int64_t(g_main_chunks.load(std::memory_order_relaxed)) << 22);
}

extern "C" int fsagg_pairgram_block8(void) {
  return g_block8.load(std::memory_order_relaxed);
}

extern "C" size_t fsagg_pairgram_workspace_bytes(int n, int64_t numel,
                                                 int nseg) {
  if (n < 2 || n > 16 * kGramMaxTiles || nseg < 1 || numel < 0) return 0;
  return gram_ws_layout(n, numel, nseg, nullptr, nullptr);
}

namespace {
int pairgram_rows(const char *what, const fsagg_rows *rows,
                  const int64_t *seg_lo, const int64_t *seg_end,
                  int64_t numel, double *segsq, double *err, double tol,
                  float *D, uint32_t *ill, float *B, double *D64,
                  void *workspace, size_t workspace_bytes,
                  fsagg_stream_t stream) {
  if (!rows || !rows->tab || !seg_lo || !seg_end || !segsq || !err ||
      rows->n < 2 || rows->n > 16 * kGramMaxTiles || rows->nseg < 1 ||
      numel < 0 || (rows->ss != 0 && rows->ss < rows->n) ||
      (D && (!ill || !(tol >= 0.0)))) {
    set_error("%s: invalid argument (n must be 2..%d)", what,
              16 * kGramMaxTiles);
    return FSAGG_EINVAL;
  }
  const int n = rows->n, nseg = rows->nseg;
  const size_t need = gram_ws_layout(n, numel, nseg, nullptr, nullptr);
  if (!workspace || workspace_bytes < need) {
    set_error("%s: workspace %zu < %zu bytes", what, workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  const GramPlan pl = gram_plan(n, numel, nseg);
  GramWs w;
  gram_ws_layout(n, numel, nseg, workspace, &w);
  hipStream_t st = as_stream(stream);
  switch (pl.nt) {
    case 1: gram_launch<1, false>(rows->tab, rows->ss, n, seg_lo, seg_end,
                                  nseg, pl, w, segsq, err, tol, D, ill, B,
                                  D64, st); break;
    case 2: gram_launch<2, false>(rows->tab, rows->ss, n, seg_lo, seg_end,
                                  nseg, pl, w, segsq, err, tol, D, ill, B,
                                  D64, st); break;
    case 3: gram_launch<3, false>(rows->tab, rows->ss, n, seg_lo, seg_end,
                                  nseg, pl, w, segsq, err, tol, D, ill, B,
                                  D64, st); break;
    case 4: gram_launch<4, false>(rows->tab, rows->ss, n, seg_lo, seg_end,
                                  nseg, pl, w, segsq, err, tol, D, ill, B,
                                  D64, st); break;
#define FSAGG_FULL(NT)                                                       \
  if (!pl.lines) {                                                           \
    gram_launch<NT, false>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg, pl, \
                           w, segsq, err, tol, D, ill, B, D64, st);          \
    break;                                                                   \
  }                                                                          \
  [[fallthrough]]
    case 5: FSAGG_FULL(5);
    case 6: FSAGG_FULL(6);
    case 7: FSAGG_FULL(7);
    case 8: FSAGG_FULL(8);
#undef FSAGG_FULL
    default:
      if (pl.nlines == 7)
        gram_launch<3, true>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg,
                             pl, w, segsq, err, tol, D, ill, B, D64, st);
      else
        gram_launch<4, true>(rows->tab, rows->ss, n, seg_lo, seg_end, nseg,
                             pl, w, segsq, err, tol, D, ill, B, D64, st);
      break;
  }
  return check_launch(what);
}
}  // namespace

extern "C" int fsagg_pairgram_rows_segsq_f32(const fsagg_rows *rows,
                                             const int64_t *seg_lo,
                                             const int64_t *seg_end,
                                             int64_t numel, double *segsq,
                                             double *err, void *workspace,
                                             size_t workspace_bytes,
                                             fsagg_stream_t stream) {
  return pairgram_rows("fsagg_pairgram_rows_segsq_f32", rows, seg_lo,
                       seg_end, numel, segsq, err, 0.0, nullptr, nullptr,
                       nullptr, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int fsagg_pairgram_rows_f32(const fsagg_rows *rows,
                                       const int64_t *seg_lo,
                                       const int64_t *seg_end, int64_t numel,
                                       double tol, double *segsq,
                                       double *err, float *D, uint32_t *ill,
                                       float *bound, double *dist64,
                                       void *workspace,
                                       size_t workspace_bytes,
                                       fsagg_stream_t stream) {
  if (!D) {
    set_error("fsagg_pairgram_rows_f32: D is NULL");
    return FSAGG_EINVAL;
  }
  return pairgram_rows("fsagg_pairgram_rows_f32", rows, seg_lo, seg_end,
                       numel, segsq, err, tol, D, ill, bound, dist64,
                       workspace, workspace_bytes, stream);
}

extern "C" int fsagg_pairgram_finish_f32(const double *segsq,
                                         const double *err, int n, int nseg,
                                         double tol, float *D, uint32_t *ill,
                                         float *bound, double *dist64,
                                         fsagg_stream_t stream) {
  if (!segsq || !err || !D || !ill || n < 2 || nseg < 1 || !(tol >= 0.0)) {
    set_error("fsagg_pairgram_finish_f32: invalid argument (n=%d nseg=%d)",
              n, nseg);
    return FSAGG_EINVAL;
  }
  hipLaunchKernelGGL(gram_finish_kernel,
                     dim3(unsigned((int64_t(n) * n + 255) / 256)), dim3(256),
                     0, as_stream(stream), segsq, err, n, nseg, tol, D, ill,
                     bound, dist64);
  return check_launch("fsagg_pairgram_finish_f32");
}
