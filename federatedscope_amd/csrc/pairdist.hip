// Krum pairwise distances and per-client norms (gfx950).
//
// Krum (krum_aggregator.py:41-77) needs, for every client pair (a, b) and
// every state_dict key, Σ_p (x_a[p] - x_b[p])^2 over the key's elements; the
// distance is the SUM over keys of the per-key L2 norms.  That is a Gram-like
// reduction over the coordinates (K = P, M = N = n) with a difference-square
// inner op; it is done on the VALU (exact fp32 differences, no MFMA: the
// ‖a‖²+‖b‖²−2a·b rewrite cancels catastrophically for near-identical
// honest clients, which is exactly the regime Krum must rank).
//
// Work decomposition
//   * the flat bucket is cut into ~1000 chunks that never straddle a key (a
//     per-key chunk prefix is built on the device); one workgroup per chunk
//     (× role groups when there are more tile pairs than threads);
//   * the chunk streams through LDS in stages of `sub` coordinates, stored
//     coordinate-major ([coord][client], row pitch ldsp); a full stage is
//     loaded with 16-B non-temporal loads into registers one stage ahead, so
//     the HBM latency hides behind the current stage's FMAs;
//   * the clients are cut into tiles of TS = 8 or 10 (whichever gives fewer
//     pair slots: at n = 50, 15 × 100 = 1500 vs 28 × 64 = 1792); each lane
//     owns one TS×TS tile pair of the upper triangle (TS² fp32 accumulators)
//     and a k-slice of the stage's coordinates; in the split-role form (the
//     default when it fits) whole waves own the off-diagonal tile pairs and
//     the others pairs of diagonal tiles, whose two upper triangles fill one
//     TS² accumulator set (n = 50: 1300 pair slots instead of 1500); at the
//     end of the chunk the k-slices are summed through LDS in a fixed order
//     → partial[chunk][pair];
//   * a 1024-thread kernel sums each key's chunks in fp64 (fixed order), and
//     a final kernel takes the per-key sqrt, rounds to fp32 and accumulates
//     the keys in fp32 in key order (the reference's
//     `distance += torch.dist(...)`).
// Deterministic: no atomics anywhere.
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>

#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;
// the staged coordinate row of every client must fit the LDS many times
// over (and the n²-sized workspace stay sane)
constexpr int kMaxPairClients = 4096;
constexpr int kPtrSlots = 512;                // LDS row-pointer table
constexpr int kRedPitch = 65;                  // LDS pitch of a reduction slot
constexpr int kLdsFloats = kBlock * kRedPitch;  // 16640 floats = 65 KiB
// register-prefetched staging items per thread (each 4 rows × 4
// coordinates); 10×10 tiles keep one fewer (their accumulators need the
// registers) and stage fewer coordinates per pass
constexpr int stage_items(int ts) { return ts == 10 ? 3 : 4; }
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

// 8×8 tiles have the registers to unroll two coordinates (the LDS latency
// of one hides behind the FMAs of the other); 10×10 do not
template <int TS>
constexpr int kCoordUnroll = TS == 8 ? 2 : 1;

// accumulator of pair (u, v) in the row-pair packed form acc[u/2][v]
template <int TS>
__device__ __forceinline__ float pair_acc(const f2 (&acc)[TS / 2][TS], int u,
                                          int v) {
  return (u & 1) ? acc[u >> 1][v].y : acc[u >> 1][v].x;
}

// Client tiles of side ts (8 or 10: the one with fewer pair slots
// ntp·ts²; at n = 50, 15 × 100 = 1500 against 28 × 64 = 1792); each lane
// accumulates one ts × ts tile pair of the upper triangle (diagonal tiles
// whole, so every lane runs the same code).
struct PairPlan {
  int ts;       // tile side
  int nt;       // tiles per side
  int ntp;      // upper-triangular tile pairs
  int groups;   // grid.y
  int tpg;      // tile pairs per group
  int ks;       // k-slices per tile pair
  int ldsp;     // LDS pitch (floats) of one staged coordinate
  int sub;      // coordinates per stage
  int64_t chl;  // coordinates per chunk
  int64_t max_chunks;
  // split-role form (split = 1): the first `wo` waves own the ro
  // off-diagonal tile pairs (kso k-slices each), the other waves the rd
  // diagonal roles — tiles 2d and 2d+1, the two upper triangles packed into
  // one TS×TS accumulator set (kso/ksd k-slices); no slot is spent on a
  // diagonal tile's lower half
  int split, wo, ro, kso, rd, ksd;
};

// The LDS pitch of a staged coordinate row: ≥ the client slots, ≡ 4 (mod
// 8) words — with the blocked item order of stage_item() (8 lanes = 2
// coordinate groups × 4 client quads) every ds_write_b128 lane group then
// hits 8 distinct 4-bank sets
inline int stage_pitch(int quads) {
  int p = quads * 4;
  while (p % 8 != 4) p += 4;
  return p;
}

PairPlan make_plan(int n, int64_t numel, int nseg) {
  PairPlan pl;
  const int nt8 = (n + 7) / 8, nt10 = (n + 9) / 10;
  pl.ts = int64_t(nt10) * (nt10 + 1) / 2 * 100 < int64_t(nt8) * (nt8 + 1) / 2 * 64
              ? 10 : 8;
  pl.nt = (n + pl.ts - 1) / pl.ts;
  pl.ntp = pl.nt * (pl.nt + 1) / 2;
  pl.groups = (pl.ntp + kBlock - 1) / kBlock;
  pl.tpg = (pl.ntp + pl.groups - 1) / pl.groups;
  pl.ks = kBlock / pl.tpg;
  pl.split = 0;
  pl.wo = pl.ro = pl.kso = pl.rd = pl.ksd = 0;
  // pitch ≡ 28 (mod 32) words: conflict-free b128 staging writes and reads
  pl.ldsp = (pl.nt * pl.ts + 3) / 4 * 4 + 4;
  while (pl.ldsp % 32 != 28) pl.ldsp += 4;
  // Stage length: a multiple of lcm(4, ks), so every k-slice gets the same
  // number of coordinates per stage (at n = 50, ks = 17: 204 coordinates,
  // 12 per lane, where 192 gave 11 or 12) and float4 rows stay whole; at
  // most what the LDS holds and, when the stage can be register-prefetched
  // (stage_items(ts) float4 quads per thread), what the registers hold.
  const int unit = std::lcm(4, pl.ks);
  // double-buffered stages: two stage buffers share the LDS (one row of
  // each buffer region stays free for the kernel's zero row)
  const int lds_cap = kLdsFloats / 2 / pl.ldsp - 1;
  const int quads = (pl.nt * pl.ts + 3) / 4;
  const int reg_cap = stage_items(pl.ts) * kBlock / quads * 4;
  const int limit = reg_cap >= unit && reg_cap < lds_cap ? reg_cap : lds_cap;
  pl.sub = limit / unit * unit;
  if (pl.sub < unit) pl.sub = limit >= 4 ? limit / 4 * 4 : limit;  // huge n
  // Split-role form, when it covers more coordinates per unit of lane time:
  // a stage costs max(⌈sub/kso⌉, ⌈sub/ksd⌉) coordinate steps of TS² packed
  // ops against ⌈sub/ks⌉ for the whole-tile form (at n = 50: 152 / 8 = 19
  // coordinates per step against 136 / 8 = 17)
  if (pl.groups == 1 && pl.nt >= 2) {
    const int ro = pl.nt * (pl.nt - 1) / 2, rd = (pl.nt + 1) / 2;
    const int ldsp = stage_pitch(quads);
    const int lcap = kLdsFloats / 2 / ldsp - 1;
    double best = double(pl.sub) / ((pl.sub + pl.ks - 1) / pl.ks) * 1.03;
    for (int wo = 1; wo < kBlock / kWave; ++wo) {
      const int kso = kWave * wo / ro, ksd = kWave * (kBlock / kWave - wo) / rd;
      if (kso < 1 || ksd < 1) continue;
      const int u = std::lcm(8, kso);  // whole float4 rows, even groups
      const int rcap = 2 * kBlock / quads * 4;  // two items per thread
      const int lim = rcap < lcap ? rcap : lcap;
      const int sub = lim / u * u;
      if (sub < u) continue;
      const int steps = std::max((sub + kso - 1) / kso, (sub + ksd - 1) / ksd);
      const double eff = double(sub) / steps;
      if (eff > best) {
        best = eff;
        pl.split = 1;
        pl.wo = wo;
        pl.ro = ro;
        pl.kso = kso;
        pl.rd = rd;
        pl.ksd = ksd;
        pl.ldsp = ldsp;
        pl.sub = sub;
      }
    }
  }
  // ≈ 1000 chunks (two rounds of the 2 × 256 resident workgroups), whole
  // stages (16-B aligned whenever the chunk start is)
  const int64_t rounds = 1024;
  const int64_t target = rounds - nseg > 256 ? rounds - nseg : 256;
  int64_t chl = (numel + target - 1) / target;
  if (chl < 2048) chl = 2048;
  pl.chl = (chl + pl.sub - 1) / pl.sub * pl.sub;
  pl.max_chunks = numel / chl + nseg + 1;
  return pl;
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Key segment s covers [seg_lo[s], seg_end[s]); the flat API passes its
// contiguous offsets as seg_lo = seg_off, seg_end = seg_off + 1.
__global__ void chunk_prefix_kernel(const int64_t *__restrict__ seg_lo,
                                    const int64_t *__restrict__ seg_end,
                                    int nseg, int64_t chl, int *prefix) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int acc = 0;
  prefix[0] = 0;
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_end[s] - seg_lo[s];
    acc += int((len + chl - 1) / chl);
    prefix[s + 1] = acc;
  }
}

__device__ __forceinline__ void tp_to_tiles(int tp, int nt, int &ti, int &tj) {
  int r = 0, base = 0;
  while (tp >= base + (nt - r)) {
    base += nt - r;
    ++r;
  }
  ti = r;
  tj = r + (tp - base);
}

// off-diagonal tile pair r (ti < tj, row-major) → tiles
__device__ __forceinline__ void od_to_tiles(int r, int nt, int &ti, int &tj) {
  int t = 0, base = 0;
  while (r >= base + (nt - 1 - t)) {
    base += nt - 1 - t;
    ++t;
  }
  ti = t;
  tj = t + 1 + (r - base);
}

// tiles (ti <= tj) → tile-pair index of tp_to_tiles
__device__ __forceinline__ int tiles_to_tp(int ti, int tj, int nt) {
  return ti * nt - ti * (ti - 1) / 2 + (tj - ti);
}

// Stage item `it` → (client quad qd, coordinate group g).  Blocks of 8
// items = 4 consecutive quads × 2 consecutive groups, so the 8 lanes of a
// ds_write_b128 group land on 8 distinct 4-bank sets (pitch ≡ 4 mod 8) and
// each 16-B row load of a wave still covers 16 consecutive groups of 4 rows;
// the quads past the last whole block of 4 (or every quad, for an odd
// group count) in plain order.
__device__ __forceinline__ void stage_item(int it, int quads, int groups,
                                           int &qd, int &g) {
  const int q4 = (groups & 1) ? 0 : quads / 4;
  const int blocked = q4 * 4 * groups;
  if (it < blocked) {
    const int half = groups >> 1;
    const int b = it >> 3, w = it & 7;
    const int qb = b / half;
    qd = 4 * qb + (w & 3);
    g = 2 * (b - qb * half) + (w >> 2);
  } else {
    const int r = it - blocked;
    const int q = r / groups;
    qd = 4 * q4 + q;
    g = r - q * groups;
  }
}

// TS values of tile t at one staged coordinate row
template <int TS>
__device__ __forceinline__ void read_tile(const float *col, int t,
                                          float (&x)[TS]) {
  if constexpr (TS % 4 == 0) {  // ds_read_b128
    const float4 *p = reinterpret_cast<const float4 *>(col + t * TS);
#pragma unroll
    for (int q = 0; q < TS / 4; ++q) {
      const float4 v = p[q];
      x[4 * q] = v.x;
      x[4 * q + 1] = v.y;
      x[4 * q + 2] = v.z;
      x[4 * q + 3] = v.w;
    }
  } else {  // ds_read_b64 (t·TS floats is 8-B aligned for even TS)
    const float2 *p = reinterpret_cast<const float2 *>(col + t * TS);
#pragma unroll
    for (int q = 0; q < TS / 2; ++q) {
      const float2 v = p[q];
      x[2 * q] = v.x;
      x[2 * q + 1] = v.y;
    }
  }
}

// One coordinate's distance updates of a lane, from its two tiles' values
// at that coordinate as row pairs (A[h] = rows 2h, 2h+1 of tile ti; B the
// same of tile tj).  Off-diagonal (DIAG false): every slot, acc[h][v] +=
// (A[h] − B_v)².  Diagonal roles (the split form's tiles ti and tj = ti+1):
// tile ti's pairs (u, v), u < v, in acc[u/2][v] (the slots 2h < v) and tile
// tj's slot (h, v) mirrored to acc[TS/2−1−h][TS−1−v] (exactly the slots
// 2h ≥ v).  All differences of a v first, then the fmas: a packed fma that
// reads the packed add just before it needs a wait state (s_nop).
template <int TS, bool DIAG>
__device__ __forceinline__ void pair_update(f2 (&acc)[TS / 2][TS],
                                            const f2 (&A)[TS / 2],
                                            const f2 (&B)[TS / 2]) {
  if constexpr (DIAG) {
#pragma unroll
    for (int v = 1; v < TS; ++v) {
      const float av = (v & 1) ? A[v >> 1].y : A[v >> 1].x;
      const float bv = (v & 1) ? B[v >> 1].y : B[v >> 1].x;
      f2 da[TS / 2], db[TS / 2];
#pragma unroll
      for (int h = 0; 2 * h < v; ++h) {
        da[h] = A[h] - f2{av, av};
        db[h] = B[h] - f2{bv, bv};
      }
#pragma unroll
      for (int h = 0; 2 * h < v; ++h) {
        acc[h][v] = __builtin_elementwise_fma(da[h], da[h], acc[h][v]);
        f2 &m = acc[TS / 2 - 1 - h][TS - 1 - v];
        m = __builtin_elementwise_fma(db[h], db[h], m);
      }
    }
  } else {
#pragma unroll
    for (int v = 0; v < TS; ++v) {
      const float bv = (v & 1) ? B[v >> 1].y : B[v >> 1].x;
      f2 d[TS / 2];
#pragma unroll
      for (int h = 0; h < TS / 2; ++h) d[h] = A[h] - f2{bv, bv};
#pragma unroll
      for (int h = 0; h < TS / 2; ++h)
        acc[h][v] = __builtin_elementwise_fma(d[h], d[h], acc[h][v]);
    }
  }
}

// The same step with its operand reads as separate ds_read_b64 (LDSR = 1):
// the compiler merges the row-pair reads into ds_read2_b64, which the LDS
// serves as 4 × 16-lane groups on 32 banks (8 cycles for 16 B per lane, 2-way
// conflicted between k-slices of the staged pitch), where two ds_read_b64 take
// 2 cycles each on 64 banks.  The reads are issued in the order the updates
// consume them and each group of updates waits only for its own (counted
// lgkmcnt; the wait names the registers it releases, so no use of them moves
// above it).  ``ca``/``cb``: LDS byte addresses of the two tiles' rows.
#define FSAGG_DSR(dst, addr, off) \
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "n"(off))
#define FSAGG_LGKM(N, a, b) \
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N))
#define FSAGG_LGKM3(N, a, b, c) \
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N))
template <int TS, bool DIAG>
__device__ __forceinline__ void pair_step_dsr(f2 (&acc)[TS / 2][TS],
                                              uint32_t ca, uint32_t cb) {
  static_assert(TS == 10, "the counted waits are written for 10-row tiles");
  f2 A[TS / 2], B[TS / 2];
  if constexpr (DIAG) {
    // A0 B0 A1 B1 ...: updates of v ∈ {2k, 2k+1} need row pairs ≤ k
    FSAGG_DSR(A[0], ca, 0);  FSAGG_DSR(B[0], cb, 0);
    FSAGG_DSR(A[1], ca, 8);  FSAGG_DSR(B[1], cb, 8);
    FSAGG_DSR(A[2], ca, 16); FSAGG_DSR(B[2], cb, 16);
    FSAGG_DSR(A[3], ca, 24); FSAGG_DSR(B[3], cb, 24);
    FSAGG_DSR(A[4], ca, 32); FSAGG_DSR(B[4], cb, 32);
  } else {
    // A0..A4 B0..B4: every update needs all of A and B[v/2]
    FSAGG_DSR(A[0], ca, 0);  FSAGG_DSR(A[1], ca, 8);
    FSAGG_DSR(A[2], ca, 16); FSAGG_DSR(A[3], ca, 24);
    FSAGG_DSR(A[4], ca, 32);
    FSAGG_DSR(B[0], cb, 0);  FSAGG_DSR(B[1], cb, 8);
    FSAGG_DSR(B[2], cb, 16); FSAGG_DSR(B[3], cb, 24);
    FSAGG_DSR(B[4], cb, 32);
  }
  // group k's wait also names an accumulator the previous group just
  // updated, so the scheduler keeps that group's updates above the wait
  auto wait_for = [&](int k) {
    // row pairs <= k of both tiles have landed
    f2 &prev = acc[0][k > 0 ? 2 * k - 1 : 0];
    if constexpr (DIAG) {
      switch (k) {
        case 0: FSAGG_LGKM(8, A[0], B[0]); break;
        case 1: FSAGG_LGKM3(6, A[1], B[1], prev); break;
        case 2: FSAGG_LGKM3(4, A[2], B[2], prev); break;
        case 3: FSAGG_LGKM3(2, A[3], B[3], prev); break;
        default: FSAGG_LGKM3(0, A[4], B[4], prev); break;
      }
    } else {
      switch (k) {
        case 0:
          FSAGG_LGKM(4, A[4], B[0]);
          asm volatile("" : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]));
          break;
        case 1: FSAGG_LGKM(3, B[1], prev); break;
        case 2: FSAGG_LGKM(2, B[2], prev); break;
        case 3: FSAGG_LGKM(1, B[3], prev); break;
        default: FSAGG_LGKM(0, B[4], prev); break;
      }
    }
  };
  if constexpr (DIAG) {
#pragma unroll
    for (int v = 1; v < TS; ++v) {
      if (v == 1 || (v & 1) == 0) wait_for(v >> 1);
      const float av = (v & 1) ? A[v >> 1].y : A[v >> 1].x;
      const float bv = (v & 1) ? B[v >> 1].y : B[v >> 1].x;
      f2 da[TS / 2], db[TS / 2];
#pragma unroll
      for (int h = 0; 2 * h < v; ++h) {
        da[h] = A[h] - f2{av, av};
        db[h] = B[h] - f2{bv, bv};
      }
#pragma unroll
      for (int h = 0; 2 * h < v; ++h) {
        acc[h][v] = __builtin_elementwise_fma(da[h], da[h], acc[h][v]);
        f2 &m = acc[TS / 2 - 1 - h][TS - 1 - v];
        m = __builtin_elementwise_fma(db[h], db[h], m);
      }
    }
  } else {
#pragma unroll
    for (int v = 0; v < TS; ++v) {
      if ((v & 1) == 0) wait_for(v >> 1);
      const float bv = (v & 1) ? B[v >> 1].y : B[v >> 1].x;
      f2 d[TS / 2];
#pragma unroll
      for (int h = 0; h < TS / 2; ++h) d[h] = A[h] - f2{bv, bv};
#pragma unroll
      for (int h = 0; h < TS / 2; ++h)
        acc[h][v] = __builtin_elementwise_fma(d[h], d[h], acc[h][v]);
    }
  }
}
#undef FSAGG_DSR
#undef FSAGG_LGKM
#undef FSAGG_LGKM3

// Partial slot of a split-form accumulator: element idx = u·TS + v of a
// lane of role `l` (off-diagonal pair l, or diagonal role l = tiles 2l,
// 2l+1) → tile pair tp and element within it; false for a slot no pair
// owns (a diagonal tile's repeated half, or a tile past the last).
__device__ __forceinline__ bool split_slot(bool diag, int l, int idx, int ts,
                                           int nt, int &tp, int &e) {
  const int u = idx / ts, v = idx % ts;
  if (!diag) {
    int a, b;
    od_to_tiles(l, nt, a, b);
    tp = tiles_to_tp(a, b, nt);
    e = idx;
    return true;
  }
  const int h = u >> 1, half = u & 1;
  int t = 2 * l, uu = u, vv = v;
  if (2 * h >= v) {  // tile B's mirrored slot
    t = 2 * l + 1;
    uu = 2 * (ts / 2 - 1 - h) + half;
    vv = ts - 1 - v;
  }
  tp = tiles_to_tp(t, t, nt);
  e = uu * ts + vv;
  return uu < vv && t < nt;
}

// Row-pair packed updates (v_pk_add_f32 / v_pk_fma_f32, two pairs per
// instruction) over double-buffered LDS stages.  SPLIT: the split-role form
// of PairPlan; LDSR = 1 reads its operands with pair_step_dsr.
template <int TS, bool SPLIT, int LDSR = 0>
__global__ __launch_bounds__(kBlock) void pairdist_chunk_kernel(
    const float *const *__restrict__ tab, int64_t ss, int n,
    PairPlan pl, const int64_t *__restrict__ seg_lo,
    const int64_t *__restrict__ seg_end, int nseg,
    const int *__restrict__ prefix, float *__restrict__ partial) {
  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
  // client row pointers for the prefetch (n <= kPtrSlots, else no
  // prefetch: stages are loaded by the scalar path): the per-lane
  // pointer gather of a stage's items then costs LDS reads, which never
  // wait behind the HBM loads already in flight (vmcnt is in order)
  __shared__ const float *rowp[kPtrSlots];
  const int c = blockIdx.x;
  const int total = prefix[nseg];
  if (c >= total) return;
  // segment s: largest s with prefix[s] <= c
  int lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= c) lo = mid;
    else hi = mid;
  }
  const int s = lo;
  const int64_t start = seg_lo[s] + int64_t(c - prefix[s]) * pl.chl;
  int64_t end = start + pl.chl;
  if (end > seg_end[s]) end = seg_end[s];
  // client r's row of this key segment: rows[r] (a virtual base)
  const float *const *__restrict__ rows = tab + int64_t(s) * ss;

  const int tid = threadIdx.x;
  int tpl = 0, ksl, kstep;
  bool active, diag = false;
  int ti = 0, tj = 0;
  bool swapped = false;  // diagonal role with its two tiles read swapped
  if constexpr (SPLIT) {
    // wave-uniform role: off-diagonal tile pairs, or diagonal tile pairs
    // (2d, 2d+1) whose two upper triangles share one accumulator set
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    diag = wave >= pl.wo;
    if (!diag) {
      ksl = tid / pl.ro;
      kstep = pl.kso;
      active = ksl < pl.kso;
      od_to_tiles(tid - ksl * pl.ro, pl.nt, ti, tj);
    } else {
      const int l = tid - kWave * pl.wo;
      ksl = l / pl.rd;
      kstep = pl.ksd;
      active = ksl < pl.ksd;
      ti = 2 * (l - ksl * pl.rd);
      tj = ti + 1 < pl.nt ? ti + 1 : ti;  // odd tile count: a repeat, unused
      // Every diagonal lane's tile ti starts at a multiple of 4 words of a
      // staged row (ti even, TS = 10, pitch ≡ 0 mod 4), so the 32 lanes of
      // a ds_read_b64 group meet only 16 bank pairs (2-way conflicts).  Lanes
      // of odd k-slices read the tiles the other way round (tile tj's rows at
      // ≡ 2 mod 4 words in the same instruction) and swap the two triangles'
      // accumulators back after the chunk (pair_update's two halves are
      // symmetric: acc[h][v] <-> acc[TS/2-1-h][TS-1-v]).
      if constexpr (LDSR == 1) {
        if (ksl & 1) {
          const int t = ti;
          ti = tj;
          tj = t;
          swapped = true;
        }
      }
    }
  } else {
    tpl = tid % pl.tpg;
    ksl = tid / pl.tpg;
    kstep = pl.ks;
    const int tp = blockIdx.y * pl.tpg + tpl;
    active = ksl < pl.ks && tpl < pl.tpg && tp < pl.ntp;
    if (active) tp_to_tiles(tp, pl.nt, ti, tj);
  }

  // client slots (rows >= n repeat row n-1), rounded to whole quads
  const int quads = (pl.nt * TS + 3) / 4;
  // A full stage is staged from registers: item = (client quad, 4
  // consecutive coordinates) = four 16-B row loads, issued for stage s + 1
  // before stage s is computed, so the HBM latency hides behind the FMAs.
  const int groups = pl.sub / 4;
  const int items = quads * groups;
  bool vec = (start & 3) == 0;
  for (int r = 0; r < n; ++r)
    vec = vec && (reinterpret_cast<uintptr_t>(rows[r]) & 15u) == 0;

  // acc[h][v] = (pair (2h, v), pair (2h+1, v)) of the tile pair: tile
  // ti's rows 2h, 2h+1 are adjacent in a staged coordinate row, so one
  // ds_read_b64 gives both and each v_pk_add_f32 / v_pk_fma_f32 works two
  // pairs with tile tj's value broadcast (op_sel) — no operand moves
  static_assert(TS % 2 == 0, "row pairs");
  f2 acc[TS / 2][TS];
#pragma unroll
  for (int h = 0; h < TS / 2; ++h)
#pragma unroll
    for (int v = 0; v < TS; ++v) acc[h][v] = f2{0.0f, 0.0f};

  // the split form keeps two stages in flight in registers (two sets of two
  // items: 64 VGPRs), the whole-tile form one stage (stage_items(TS) items)
  constexpr int kStageItems = SPLIT ? 2 : stage_items(TS);
  f4v pre[kStageItems][4], pre1[kStageItems][4];
  // global (not flat) loads: a flat load also counts in lgkmcnt, so the
  // compute loop's first LDS-read wait would wait for the whole prefetch
  typedef __attribute__((address_space(1))) const f4v gf4v;
  // this thread's stage items, placed once (qd < 0: none)
  // (the split form's loads are issued by every lane, a lane without item k
  // re-reading the last item: no branch around a load, so the compiler's
  // vmcnt bookkeeping stays exact and a stage waits only for its own set)
  int item_qd[kStageItems], item_g[kStageItems];
  bool item_ok[kStageItems];
#pragma unroll
  for (int k = 0; k < kStageItems; ++k) {
    const int it = tid + k * kBlock;
    item_ok[k] = it < items;
    stage_item(it < items ? it : items - 1, quads, groups, item_qd[k],
               item_g[k]);
  }
  auto fetch = [&](int64_t cs, f4v (&pre)[kStageItems][4]) {
#pragma unroll
    for (int k = 0; k < kStageItems; ++k) {
      if (SPLIT || item_ok[k]) {
        const int qd = item_qd[k], g = item_g[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = min(qd * 4 + e, n - 1);
          const float *row = rowp[r];
          pre[k][e] = __builtin_nontemporal_load(
              (gf4v *)(row + cs) + g);
        }
      }
    }
  };
  auto stage_from_regs = [&](float *buf, const f4v (&pre)[kStageItems][4]) {
#pragma unroll
    for (int k = 0; k < kStageItems; ++k) {
      if (item_ok[k]) {
        const int qd = item_qd[k], g = item_g[k];
        float *dst = buf + (4 * g) * pl.ldsp + qd * 4;
        *reinterpret_cast<float4 *>(dst) =
            make_float4(pre[k][0].x, pre[k][1].x, pre[k][2].x, pre[k][3].x);
        *reinterpret_cast<float4 *>(dst + pl.ldsp) =
            make_float4(pre[k][0].y, pre[k][1].y, pre[k][2].y, pre[k][3].y);
        *reinterpret_cast<float4 *>(dst + 2 * pl.ldsp) =
            make_float4(pre[k][0].z, pre[k][1].z, pre[k][2].z, pre[k][3].z);
        *reinterpret_cast<float4 *>(dst + 3 * pl.ldsp) =
            make_float4(pre[k][0].w, pre[k][1].w, pre[k][2].w, pre[k][3].w);
      }
    }
  };
  // partial or unaligned stage: guarded 4-B loads straight to LDS
  auto stage_scalar = [&](float *buf, int64_t cs, int len) {
    const int wave = tid / kWave, lane = tid & (kWave - 1);
    for (int qd = wave; qd < quads; qd += kBlock / kWave) {
      const int r0 = qd * 4;
      const float *p0 = rows[min(r0, n - 1)] + cs;
      const float *p1 = rows[min(r0 + 1, n - 1)] + cs;
      const float *p2 = rows[min(r0 + 2, n - 1)] + cs;
      const float *p3 = rows[min(r0 + 3, n - 1)] + cs;
      for (int cc = lane; cc < len; cc += kWave)
        *reinterpret_cast<float4 *>(buf + cc * pl.ldsp + r0) =
            make_float4(gld(p0 + cc), gld(p1 + cc), gld(p2 + cc), gld(p3 + cc));
    }
  };

  const bool prefetch =
      vec && items <= kStageItems * kBlock && n <= kPtrSlots;
  // a zero row past the last stage row of buffer 0 (the plan keeps it
  // free): lanes past their last coordinate of a stage read it
  float *const zrow = lds + kLdsFloats / 2 - pl.ldsp;
  for (int i = tid; i < pl.ldsp; i += kBlock) zrow[i] = 0.0f;
  if (n <= kPtrSlots) {
    for (int r = tid; r < n; r += kBlock) rowp[r] = rows[r];
  }
  __syncthreads();
  // one stage's distance updates from the staged rows in buf
  // role: std::true_type for the diagonal roles of the split form
  // A wave-uniform trip count (len and kstep are): a lane past its last
  // coordinate, or an idle lane, reads the zero row and adds (0 - 0)^2 — no
  // divergent loop, so the accumulators stay in place across stages.
  auto compute = [&](const float *buf, int len, auto role) {
    const int steps = (len + kstep - 1) / kstep;
    auto col_of = [&](int s) {
      const int cc = ksl + s * kstep;
      return active && cc < len ? buf + cc * pl.ldsp : zrow;
    };
    if constexpr (SPLIT) {
      auto load = [&](int s, f2 (&A)[TS / 2], f2 (&B)[TS / 2]) {
        const float *col = col_of(s);
        const f2 *pa = reinterpret_cast<const f2 *>(col + ti * TS);
        const f2 *pb = reinterpret_cast<const f2 *>(col + tj * TS);
#pragma unroll
        for (int h = 0; h < TS / 2; ++h) {
          A[h] = pa[h];
          B[h] = pb[h];
        }
      };
      int s = 0;
      if constexpr (LDSR == 1) {
        typedef __attribute__((address_space(3))) const float lds_f;
        auto at = [](const float *p) {
          return uint32_t(uintptr_t((lds_f *)p));
        };
        // every coordinate ksl + s·kstep of the first len / kstep steps
        // lies inside the stage: those steps take no zero-row select, only
        // an address increment (idle lanes read the zero row throughout)
        const int plain = len / kstep;  // wave-uniform
        if (plain > 0) {
          const float *col = active ? buf + ksl * pl.ldsp : zrow;
          uint32_t ca = at(col + ti * TS), cb = at(col + tj * TS);
          const uint32_t inc = active ? uint32_t(kstep * pl.ldsp * 4) : 0u;
          do {
            pair_step_dsr<TS, decltype(role)::value>(acc, ca, cb);
            ca += inc;
            cb += inc;
          } while (++s < plain);
        }
        for (; s < steps; ++s) {
          const float *col = col_of(s);
          pair_step_dsr<TS, decltype(role)::value>(acc, at(col + ti * TS),
                                                   at(col + tj * TS));
        }
        return;
      }
      do {  // len >= 1: at least one step
        f2 A[TS / 2], B[TS / 2];
        load(s, A, B);
        pair_update<TS, decltype(role)::value>(acc, A, B);
      } while (++s < steps);
      return;
    }
#pragma unroll kCoordUnroll<TS>
    for (int s = 0; s < steps; ++s) {
      const float *col = col_of(s);
      float b[TS];
      read_tile<TS>(col, tj, b);
      const f2 *ap = reinterpret_cast<const f2 *>(col + ti * TS);
      f2 a[TS / 2];
#pragma unroll
      for (int h = 0; h < TS / 2; ++h) a[h] = ap[h];
#pragma unroll
      for (int v = 0; v < TS; ++v) {
        // all TS/2 differences first, then the fmas: a packed fma that
        // reads the packed add just before it needs a wait state (s_nop)
        f2 d[TS / 2];
#pragma unroll
        for (int h = 0; h < TS / 2; ++h) d[h] = a[h] - f2{b[v], b[v]};
#pragma unroll
        for (int h = 0; h < TS / 2; ++h)
          acc[h][v] = __builtin_elementwise_fma(d[h], d[h], acc[h][v]);
      }
    }
  };
  auto stage_len = [&](int64_t cs) {
    return int(end - cs < pl.sub ? end - cs : pl.sub);
  };

  // the stage loop, instantiated per role (a wave-uniform branch around
  // whole loops: the accumulators merge once, after the chunk)
  auto run = [&](auto role) {
  if constexpr (SPLIT) {
    // Two stages in flight: the rows of stage s + 2 are loaded into the
    // register set stage s + 1 was just staged from, so each load has two
    // stages of distance updates to land.  Unrolled by two: sets pre (even
    // stages) and pre1 (odd) are fixed registers.  Every trip issues its
    // loads (clamped to the chunk's last whole stage near its end).
    float *const buf0 = lds, *const buf1 = lds + kLdsFloats / 2;
    if (prefetch && end - start >= pl.sub) {
      const int64_t last = start + ((end - pl.sub - start) & ~int64_t(3));
      auto fetch_at = [&](int64_t cs, f4v (&p)[kStageItems][4]) {
        fetch(cs < last ? cs : last, p);
      };
      auto put = [&](float *buf, int64_t cs,
                     const f4v (&p)[kStageItems][4]) {
        if (end - cs >= pl.sub) stage_from_regs(buf, p);
        else stage_scalar(buf, cs, stage_len(cs));
      };
      fetch_at(start, pre);
      fetch_at(start + pl.sub, pre1);
      put(buf0, start, pre);
      fetch_at(start + 2 * pl.sub, pre);
      __syncthreads();
      for (int64_t cs = start; cs < end;) {
        int64_t ncs = cs + pl.sub;
        if (ncs < end) put(buf1, ncs, pre1);
        fetch_at(ncs + 2 * pl.sub, pre1);
        compute(buf0, stage_len(cs), role);
        __syncthreads();
        cs = ncs;
        if (cs >= end) break;
        ncs = cs + pl.sub;
        if (ncs < end) put(buf0, ncs, pre);
        fetch_at(ncs + 2 * pl.sub, pre);
        compute(buf1, stage_len(cs), role);
        __syncthreads();
        cs = ncs;
      }
    } else {
      // unaligned rows or a chunk shorter than a stage: scalar staging
      int st = 0;
      if (start < end) stage_scalar(buf0, start, stage_len(start));
      __syncthreads();
      for (int64_t cs = start; cs < end; cs += pl.sub, st ^= 1) {
        const int64_t ncs = cs + pl.sub;
        if (ncs < end) stage_scalar(st ? buf0 : buf1, ncs, stage_len(ncs));
        compute(st ? buf1 : buf0, stage_len(cs), role);
        __syncthreads();
      }
    }
    return;
  }
  if (prefetch && end - start >= pl.sub) fetch(start, pre);
  {
    // two stage buffers, one barrier per stage: stage s + 1 is written into
    // the buffer stage s - 1 was read from (every wave has passed the
    // barrier after it) while stage s is computed from the other
    auto buf_of = [&](int b) { return b ? lds + kLdsFloats / 2 : lds; };
    if (start < end) {
      const int len = stage_len(start);
      if (prefetch && len == pl.sub) stage_from_regs(lds, pre);
      else stage_scalar(lds, start, len);
    }
    __syncthreads();
    if (prefetch && end - (start + pl.sub) >= pl.sub) fetch(start + pl.sub, pre);
    int st = 0;
    for (int64_t cs = start; cs < end; cs += pl.sub, st ^= 1) {
      const int64_t ncs = cs + pl.sub;
      if (ncs < end) {
        const int nlen = stage_len(ncs);
        if (prefetch && nlen == pl.sub) stage_from_regs(buf_of(st ^ 1), pre);
        else stage_scalar(buf_of(st ^ 1), ncs, nlen);
        if (prefetch && end - (ncs + pl.sub) >= pl.sub) fetch(ncs + pl.sub, pre);
      }
      compute(buf_of(st), stage_len(cs), role);
      __syncthreads();
    }
  }
  };
  if (SPLIT && diag) run(std::true_type{});
  else run(std::false_type{});
  if constexpr (SPLIT && LDSR == 1) {
    // the swapped diagonal lanes' triangles back into place
#pragma unroll
    for (int h = 0; h < TS / 2; ++h)
#pragma unroll
      for (int v = 2 * h + 1; v < TS; ++v) {
        const f2 a = acc[h][v], b = acc[TS / 2 - 1 - h][TS - 1 - v];
        acc[h][v] = swapped ? b : a;
        acc[TS / 2 - 1 - h][TS - 1 - v] = swapped ? a : b;
      }
  }

  // sum the k-slices of each tile pair in slice order, ≤ 64 accumulators
  // at a time through LDS
  constexpr int kE = TS * TS;
  if constexpr (SPLIT) {
    // lane tid's accumulators at slot tid; role l's k-slices are lanes
    // k·ro + l (off-diagonal) or 64·wo + k·rd + d (diagonal)
#pragma unroll
    for (int e0 = 0; e0 < kE; e0 += 64) {
      const int ne = kE - e0 < 64 ? kE - e0 : 64;
      if (active) {
        float *slot = lds + tid * kRedPitch;
#pragma unroll
        for (int e = e0; e < e0 + 64 && e < kE; ++e)
          slot[e - e0] = pair_acc<TS>(acc, e / TS, e % TS);
      }
      __syncthreads();
      const int nod = pl.ro * ne;
      const int outs = nod + pl.rd * ne;
      for (int o = tid; o < outs; o += kBlock) {
        float sum = 0.0f;
        int tp, idx;
        bool valid;
        if (o < nod) {
          const int l = o / ne, e = o - l * ne;
          for (int k = 0; k < pl.kso; ++k)
            sum += lds[(k * pl.ro + l) * kRedPitch + e];
          valid = split_slot(false, l, e0 + e, TS, pl.nt, tp, idx);
        } else {
          const int o2 = o - nod;
          const int d = o2 / ne, e = o2 - d * ne;
          for (int k = 0; k < pl.ksd; ++k)
            sum += lds[(kWave * pl.wo + k * pl.rd + d) * kRedPitch + e];
          valid = split_slot(true, d, e0 + e, TS, pl.nt, tp, idx);
        }
        if (valid) partial[(int64_t(c) * pl.ntp + tp) * kE + idx] = sum;
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int e0 = 0; e0 < kE; e0 += 64) {
    if (ksl < pl.ks) {
      float *slot = lds + (ksl * pl.tpg + tpl) * kRedPitch;
#pragma unroll
      for (int e = e0; e < e0 + 64 && e < kE; ++e)
        slot[e - e0] = pair_acc<TS>(acc, e / TS, e % TS);
    }
    __syncthreads();
    const int ne = kE - e0 < 64 ? kE - e0 : 64;
    const int outs = pl.tpg * ne;
    for (int o = tid; o < outs; o += kBlock) {
      const int l = o / ne;
      const int e = o - l * ne;
      const int gtp = blockIdx.y * pl.tpg + l;
      if (gtp >= pl.ntp) continue;
      float sum = 0.0f;
      for (int k = 0; k < pl.ks; ++k)
        sum += lds[(k * pl.tpg + l) * kRedPitch + e];
      partial[(int64_t(c) * pl.ntp + gtp) * kE + e0 + e] = sum;
    }
    __syncthreads();
  }
}

// Σ over a segment's chunks in fp64 for every pair of the tile layout, in a
// fixed order (deterministic, no atomics).  Block = (segment, 64 partial
// columns); its 16 waves take every 16th chunk each (consecutive lanes read
// consecutive partials of one chunk: coalesced), then the 16 slice sums are
// added in slice order.  Output: the full symmetric [nseg][n][n] matrix of
// per-key squared distances (diagonal 0).
constexpr int kSegBlock = 1024;
constexpr int kSegSlices = kSegBlock / kWave;

__global__ __launch_bounds__(kSegBlock) void pairdist_segsq_kernel(
    const float *__restrict__ partial, int n, PairPlan pl, int nseg,
    const int *__restrict__ prefix, double *__restrict__ segsq) {
  __shared__ double red[kSegSlices][kWave];
  const int s = blockIdx.x;
  const int ee = pl.ts * pl.ts;
  const int per_seg = pl.ntp * ee;
  const int lane = threadIdx.x & (kWave - 1), slice = threadIdx.x / kWave;
  const int r = blockIdx.y * kWave + lane;
  int i = n, j = n;  // the pair of slot r (only i < j < n is ever written)
  if (r < per_seg) {
    const int tp = r / ee, e = r % ee;
    int ti, tj;
    tp_to_tiles(tp, pl.nt, ti, tj);
    i = ti * pl.ts + e / pl.ts;
    j = tj * pl.ts + e % pl.ts;
  }
  const bool want = i < j && j < n;
  double sq = 0.0;
  if (want) {
#pragma unroll 4
    for (int c = prefix[s] + slice; c < prefix[s + 1]; c += kSegSlices)
      sq += double(partial[int64_t(c) * per_seg + r]);
  }
  red[slice][lane] = sq;
  __syncthreads();
  if (slice != 0 || r >= per_seg) return;
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kSegSlices; ++k) t += red[k][lane];
  double *m = segsq + int64_t(s) * n * n;
  if (i == 0 && j == 1) {
    // the diagonal of this segment (one writer per segment)
    for (int d = 0; d < n; ++d) m[int64_t(d) * n + d] = 0.0;
  }
  if (!want) return;
  m[int64_t(i) * n + j] = t;
  m[int64_t(j) * n + i] = t;
}

// D[a][b] = Σ_seg fl32(sqrt(segsq[seg][a][b])) accumulated in fp32 in key
// order (the reference's `distance += torch.dist(...)`), D[a][a] = +inf.
__global__ __launch_bounds__(kBlock) void pairdist_finish_kernel(
    const double *__restrict__ segsq, int n, int nseg, float *__restrict__ D) {
  const int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= n * n) return;
  if (q / n == q % n) {
    D[q] = __builtin_inff();
    return;
  }
  float dist = 0.0f;
  for (int s = 0; s < nseg; ++s)
    dist = add_rn(dist, float(sqrt(segsq[int64_t(s) * n * n + q])));
  D[q] = dist;
}

// ---- per-row squared norms (fp64, deterministic) -------------------------
inline int rownorm_blocks(int n, int64_t numel) {
  int64_t b = (numel + kBlock * 16 - 1) / (kBlock * 16);
  int64_t cap = (2048 + n - 1) / n;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return int(b);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

__global__ __launch_bounds__(kBlock) void rownorm_partial_kernel(
    const float *const *__restrict__ rows, int64_t numel, int nblk,
    double *__restrict__ partial) {
  __shared__ double red[kBlock / kWave];
  const int row = blockIdx.y;
  const int64_t chunk = (numel + nblk - 1) / nblk;
  const int64_t lo = int64_t(blockIdx.x) * chunk;
  int64_t hi = lo + chunk;
  if (hi > numel) hi = numel;
  const float *x = rows[row] + lo;
  const int64_t len = hi > lo ? hi - lo : 0;
  // unguarded groups of 8 coordinates per lane (all loads issued before
  // the first use), then a guarded tail
  constexpr int G = 8;
  const int64_t full = len / (G * kBlock) * (G * kBlock);
  double acc = 0.0;
  int64_t q = threadIdx.x;
  for (; q < full; q += G * kBlock) {
    float v[G];
#pragma unroll
    for (int e = 0; e < G; ++e) v[e] = gload_nt(x + q + e * kBlock);
#pragma unroll
    for (int e = 0; e < G; ++e) acc += double(v[e]) * double(v[e]);
  }
  for (; q < len; q += kBlock) {
    const double d = double(gld(x + q));
    acc += d * d;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) t += red[w];
    partial[int64_t(row) * nblk + blockIdx.x] = t;
  }
}

__global__ void rownorm_final_kernel(const double *__restrict__ partial, int n,
                                     int nblk, double *__restrict__ sq) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  double t = 0.0;
  for (int b = 0; b < nblk; ++b) t += partial[int64_t(row) * nblk + b];
  sq[row] = t;
}

// ---- per-(client, key) squared norms over a row set (fp64) --------------
// Block (c, i) sums chunk c of client i (fixed lane order + one LDS tree) →
// partial[i][c]; then one lane per client adds its chunks in chunk order
// into sq[i][seg].  NULL entries (absent keys) contribute nothing.
__global__ __launch_bounds__(kBlock) void rows_sqnorm_partial_kernel(
    const float *const *__restrict__ tab, int64_t ss,
    const fsagg_chunk *__restrict__ chunks, int nchunk,
    double *__restrict__ partial) {
  __shared__ double red[kBlock / kWave];
  const int c = blockIdx.x, i = blockIdx.y;
  const int64_t lo = chunks[c].lo;
  const int len = chunks[c].len;
  const float *row = tab[int64_t(chunks[c].seg) * ss + i];
  double acc = 0.0;
  if (row) {
    constexpr int G = 8;
    int q = threadIdx.x;
    for (; q + (G - 1) * kBlock < len; q += G * kBlock) {
      float v[G];
#pragma unroll
      for (int e = 0; e < G; ++e) v[e] = gload_nt(row + lo + q + e * kBlock);
#pragma unroll
      for (int e = 0; e < G; ++e) acc += double(v[e]) * double(v[e]);
    }
    for (; q < len; q += kBlock) {
      const double d = double(gld(row + lo + q));
      acc += d * d;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) t += red[w];
    partial[int64_t(i) * nchunk + c] = t;
  }
}

// One wave per (client, segment): the segment's chunks are contiguous in
// the table (built key by key) — binary-search the first, lane l adds
// chunks first + l, first + l + 64, … in order, then a fixed shuffle tree.
__global__ __launch_bounds__(kBlock) void rows_sqnorm_final_kernel(
    const fsagg_chunk *__restrict__ chunks, int nchunk, int n, int nseg,
    const double *__restrict__ partial, double *__restrict__ sq) {
  const int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (q >= int64_t(n) * nseg) return;  // whole waves leave together
  const int i = int(q / nseg), s = int(q % nseg);
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
  const double *row = partial + int64_t(i) * nchunk;
  for (int c = lo + lane; c < end; c += kWave) t += row[c];
  t = wave_sum(t);
  if (lane == 0) sq[q] = t;
}

// One lane per client: the norm bounding rate from its per-key squared
// norms (normbounding_aggregator.py:39-40).  norm = fl32(sqrt(Σ_s sq)) as
// torch.norm returns it; the test `norm > bound` is fp32 against fp32 (a
// 0-dim fp32 tensor against a Python float); the rate bound / norm is
// Tensor.__rtruediv__ = fl32(fl32(1 / norm) · bound).  Unscaled clients get
// 1.0 (fl32(x · 1) = x in the weighted sum's prescale).  fp32 division and
// fp64 sqrt are correctly rounded (hipcc's defaults).
__global__ __launch_bounds__(kBlock) void normbound_prescale_kernel(
    const double *__restrict__ sq, int n, int nseg, float bound,
    float *__restrict__ prescale) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double t = 0.0;
  for (int s = 0; s < nseg; ++s) t += sq[int64_t(i) * nseg + s];
  const float norm = float(sqrt(t));
  prescale[i] = norm > bound ? (1.0f / norm) * bound : 1.0f;
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" size_t fsagg_rows_sqnorm_workspace_bytes(int n, int nchunk) {
  if (n < 1 || nchunk < 1) return 0;
  return sizeof(double) * size_t(n) * size_t(nchunk);
}

extern "C" int fsagg_rows_sqnorm_f32(const fsagg_rows *rows,
                                     const fsagg_chunk *chunks, int nchunk,
                                     double *sq, void *workspace,
                                     size_t workspace_bytes,
                                     fsagg_stream_t stream) {
  if (!rows || !rows->tab || rows->n < 1 || rows->n > 65535 ||
      rows->nseg < 1 || !sq || nchunk < 0 || (nchunk > 0 && !chunks)) {
    set_error("fsagg_rows_sqnorm_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_rows_sqnorm_workspace_bytes(rows->n, nchunk);
  if (need && (!workspace || workspace_bytes < need)) {
    set_error("fsagg_rows_sqnorm_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  double *partial = static_cast<double *>(workspace);
  if (nchunk > 0)
    hipLaunchKernelGGL(rows_sqnorm_partial_kernel,
                       dim3(unsigned(nchunk), unsigned(rows->n)), dim3(kBlock),
                       0, s, rows->tab, rows->ss, chunks, nchunk, partial);
  const int64_t waves = int64_t(rows->n) * rows->nseg;
  const int64_t per = kBlock / kWave;
  hipLaunchKernelGGL(rows_sqnorm_final_kernel,
                     dim3(unsigned((waves + per - 1) / per)), dim3(kBlock), 0,
                     s, chunks, nchunk, rows->n, rows->nseg, partial, sq);
  return check_launch("fsagg_rows_sqnorm_f32");
}

extern "C" int fsagg_normbound_prescale_f32(const double *sq, int n, int nseg,
                                            float bound, float *prescale,
                                            fsagg_stream_t stream) {
  if (!sq || !prescale || n < 1 || nseg < 1) {
    set_error("fsagg_normbound_prescale_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  hipLaunchKernelGGL(normbound_prescale_kernel,
                     dim3(unsigned((n + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, as_stream(stream), sq, n, nseg, bound, prescale);
  return check_launch("fsagg_normbound_prescale_f32");
}

// chunks of the partial buffer
static int64_t pairdist_max_chunks(int n, int64_t numel, int nseg) {
  return make_plan(n, numel, nseg).max_chunks;
}

static size_t partial_bytes(int n, int64_t numel, int nseg) {
  const PairPlan pl = make_plan(n, numel, nseg);
  return align256(sizeof(float) * size_t(pairdist_max_chunks(n, numel, nseg)) *
                  size_t(pl.ntp) * size_t(pl.ts * pl.ts));
}

// The chunk length the distance kernels plan for (n, numel, nseg): every
// fp32 partial of a pair sums at most this many squared differences (a
// k-slice's coordinates, then the slices), which bounds its rounding.
extern "C" int64_t fsagg_pairdist_chunk_elems(int n, int64_t numel,
                                              int nseg) {
  if (n < 1 || nseg < 1 || numel < 0) return 0;
  return make_plan(n, numel, nseg).chl;
}

extern "C" size_t fsagg_pairdist_workspace_bytes(int n, int64_t numel,
                                                 int nseg) {
  if (n < 1 || nseg < 1) return 0;
  return align256(sizeof(int) * size_t(nseg + 1)) +
         partial_bytes(n, numel, nseg) +
         align256(sizeof(double) * size_t(nseg) * size_t(n) * size_t(n));
}

// Enqueue the chunk and per-segment kernels; segsq receives [nseg][n][n].
static int pairdist_segsq_impl(const float *const *tab, int64_t ss, int n,
                               int64_t numel,
                               const int64_t *seg_lo, const int64_t *seg_end,
                               int nseg, double *segsq, void *workspace,
                               hipStream_t s) {
  const PairPlan pl = make_plan(n, numel, nseg);
  int *prefix = static_cast<int *>(workspace);
  float *partial = reinterpret_cast<float *>(
      static_cast<char *>(workspace) + align256(sizeof(int) * size_t(nseg + 1)));
  hipLaunchKernelGGL(chunk_prefix_kernel, dim3(1), dim3(1), 0, s, seg_lo,
                     seg_end, nseg, pl.chl, prefix);
  if (numel > 0) {
    const dim3 grid(unsigned(pl.max_chunks), unsigned(pl.groups));
#define FSAGG_CHUNK(TS, SPLIT, LDSR)                                         \
  hipLaunchKernelGGL((pairdist_chunk_kernel<TS, SPLIT, LDSR>), grid,        \
                     dim3(kBlock), 0, s, tab, ss, n, pl, seg_lo, seg_end,   \
                     nseg, prefix, partial)
    if (pl.split) {
      if (pl.ts == 10) FSAGG_CHUNK(10, true, 1);
      else FSAGG_CHUNK(8, true, 0);
    } else if (pl.ts == 10) {
      FSAGG_CHUNK(10, false, 0);
    } else {
      FSAGG_CHUNK(8, false, 0);
    }
#undef FSAGG_CHUNK
  }
  const int per_seg = pl.ntp * pl.ts * pl.ts;
  hipLaunchKernelGGL(pairdist_segsq_kernel,
                     dim3(unsigned(nseg), unsigned((per_seg + kWave - 1) / kWave)),
                     dim3(kSegBlock), 0, s, partial, n, pl, nseg, prefix, segsq);
  return FSAGG_OK;
}

extern "C" int fsagg_pairdist_f32(const float *const *rows, int n,
                                  int64_t numel, const int64_t *seg_off,
                                  int nseg, float *D, void *workspace,
                                  size_t workspace_bytes,
                                  fsagg_stream_t stream) {
  if (!rows || !seg_off || !D || n < 2 || n > kMaxPairClients ||
      nseg < 1 || numel < 0) {
    set_error("fsagg_pairdist_f32: invalid argument (n=%d nseg=%d)", n, nseg);
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_pairdist_workspace_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_pairdist_f32: workspace %zu < %zu bytes", workspace_bytes,
              need);
    return FSAGG_ESPACE;
  }
  hipStream_t s = as_stream(stream);
  double *segsq = reinterpret_cast<double *>(
      static_cast<char *>(workspace) + align256(sizeof(int) * size_t(nseg + 1)) +
      partial_bytes(n, numel, nseg));
  pairdist_segsq_impl(rows, 0, n, numel, seg_off, seg_off + 1, nseg, segsq,
                      workspace, s);
  hipLaunchKernelGGL(pairdist_finish_kernel,
                     dim3(unsigned((n * n + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, s, segsq, n, nseg, D);
  return check_launch("fsagg_pairdist_f32");
}

extern "C" int fsagg_pairdist_segsq_f32(const float *const *rows, int n,
                                        int64_t numel, const int64_t *seg_off,
                                        int nseg, double *segsq,
                                        void *workspace,
                                        size_t workspace_bytes,
                                        fsagg_stream_t stream) {
  if (!rows || !seg_off || !segsq || n < 2 || n > kMaxPairClients ||
      nseg < 1 || numel < 0) {
    set_error("fsagg_pairdist_segsq_f32: invalid argument (n=%d nseg=%d)", n,
              nseg);
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_pairdist_workspace_bytes(n, numel, nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_pairdist_segsq_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  pairdist_segsq_impl(rows, 0, n, numel, seg_off, seg_off + 1, nseg, segsq,
                      workspace, as_stream(stream));
  return check_launch("fsagg_pairdist_segsq_f32");
}

extern "C" int fsagg_pairdist_rows_segsq_f32(const fsagg_rows *rows,
                                             const int64_t *seg_lo,
                                             const int64_t *seg_end,
                                             int64_t numel, double *segsq,
                                             void *workspace,
                                             size_t workspace_bytes,
                                             fsagg_stream_t stream) {
  if (!rows || !rows->tab || !seg_lo || !seg_end || !segsq || rows->n < 2 ||
      rows->n > kMaxPairClients || rows->nseg < 1 || numel < 0) {
    set_error("fsagg_pairdist_rows_segsq_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  const size_t need =
      fsagg_pairdist_workspace_bytes(rows->n, numel, rows->nseg);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_pairdist_rows_segsq_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  pairdist_segsq_impl(rows->tab, rows->ss, rows->n, numel, seg_lo,
                      seg_end, rows->nseg, segsq, workspace,
                      as_stream(stream));
  return check_launch("fsagg_pairdist_rows_segsq_f32");
}

extern "C" int fsagg_pairdist_finish_f64(const double *segsq, int n, int nseg,
                                         float *D, fsagg_stream_t stream) {
  if (!segsq || !D || n < 2 || nseg < 1) {
    set_error("fsagg_pairdist_finish_f64: invalid argument");
    return FSAGG_EINVAL;
  }
  hipLaunchKernelGGL(pairdist_finish_kernel,
                     dim3(unsigned((n * n + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, as_stream(stream), segsq, n, nseg, D);
  return check_launch("fsagg_pairdist_finish_f64");
}

extern "C" size_t fsagg_rownorm_workspace_bytes(int n, int64_t numel) {
  if (n < 1) return 0;
  return sizeof(double) * size_t(n) * size_t(rownorm_blocks(n, numel));
}

extern "C" int fsagg_row_sqnorm_f32(const float *const *rows, int n,
                                    int64_t numel, double *sq, void *workspace,
                                    size_t workspace_bytes,
                                    fsagg_stream_t stream) {
  if (!rows || !sq || n < 1 || numel < 0) {
    set_error("fsagg_row_sqnorm_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  const size_t need = fsagg_rownorm_workspace_bytes(n, numel);
  if (!workspace || workspace_bytes < need) {
    set_error("fsagg_row_sqnorm_f32: workspace %zu < %zu bytes",
              workspace_bytes, need);
    return FSAGG_ESPACE;
  }
  const int nblk = rownorm_blocks(n, numel);
  hipStream_t s = as_stream(stream);
  double *partial = static_cast<double *>(workspace);
  hipLaunchKernelGGL(rownorm_partial_kernel, dim3(unsigned(nblk), unsigned(n)),
                     dim3(kBlock), 0, s, rows, numel, nblk, partial);
  hipLaunchKernelGGL(rownorm_final_kernel, dim3(unsigned((n + 63) / 64)),
                     dim3(64), 0, s, partial, n, nblk, sq);
  return check_launch("fsagg_row_sqnorm_f32");
}
