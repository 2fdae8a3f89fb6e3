// Probe (tools/ only, never in libfsagg): the arithmetic of gfx950's
// v_mfma_f32_16x16x32_bf16 — how a 32-product dot plus the fp32 accumulator
// is rounded — and the per-k-step error of pairgram.hip's bf16-limb Gram
// step (split into three limbs, six chained MFMAs).  tools/probe/
// mfma_numerics.py feeds adversarial inputs and compares with exact sums.
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC mfma_numerics.hip -o ...
#include <hip/hip_runtime.h>

#include <cstdint>

typedef short frag8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// One wave per case.  A [case][16][32], B [case][32][16] bf16 bits, C, D
// [case][16][16] fp32.  Lane l: A row l & 15, k = 8(l >> 4) .. +7; B column
// l & 15, same k; D rows 4(l >> 4) + r, column l & 15.
__global__ void raw_kernel(const uint16_t *A, const uint16_t *B,
                           const float *C, float *D, int ncase) {
  const int c = blockIdx.x;
  if (c >= ncase) return;
  const int l = threadIdx.x, g = l >> 4, i = l & 15;
  frag8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = short(A[(int64_t(c) * 16 + i) * 32 + 8 * g + j]);
    b[j] = short(B[(int64_t(c) * 32 + 8 * g + j) * 16 + i]);
  }
  f32x4 x;
  for (int r = 0; r < 4; ++r) x[r] = C[(int64_t(c) * 16 + 4 * g + r) * 16 + i];
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, x, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(int64_t(c) * 16 + 4 * g + r) * 16 + i] = x[r];
}

__device__ __forceinline__ uint32_t pk_rne(float a, float b) {
  return __builtin_bit_cast(uint32_t,
                            __builtin_convertvector(f32x2{a, b}, bf16x2));
}
struct Neg {
  uint32_t lo, hi;
};
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
__device__ void split3(const float (&x)[8], const Neg &k, frag8 &h, frag8 &m,
                       frag8 &lo) {
  u32x4 ph, pm, pl;
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
  lo = __builtin_bit_cast(frag8, pl);
}

// pairgram.hip's k-step: XA, XB [case][16][32] fp32 rows (16 clients x 32
// coordinates each); G [case][16][16] = Σ_k XA[i][k]·XB[j][k] through three
// limbs and six chained MFMAs (mm, hl, lh, hm, mh, hh), as the product does.
__global__ void kstep_kernel(const float *XA, const float *XB, float *G,
                             int ncase) {
  const int c = blockIdx.x;
  if (c >= ncase) return;
  const int l = threadIdx.x, g = l >> 4, i = l & 15;
  Neg kn{0x0000bf80u, 0xbf800000u};
  asm volatile("" : "+v"(kn.lo), "+v"(kn.hi));
  float xa[8], xb[8];
  for (int j = 0; j < 8; ++j) {
    const int k = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
    xa[j] = XA[(int64_t(c) * 16 + i) * 32 + k];
    xb[j] = XB[(int64_t(c) * 16 + i) * 32 + k];
  }
  frag8 ha, ma, la, hb, mb, lb;
  split3(xa, kn, ha, ma, la);
  split3(xb, kn, hb, mb, lb);
  f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ma, mb, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha, lb, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(la, hb, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha, mb, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ma, hb, x, 0, 0, 0);
  x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha, hb, x, 0, 0, 0);
  for (int r = 0; r < 4; ++r) G[(int64_t(c) * 16 + 4 * g + r) * 16 + i] = x[r];
}

extern "C" int probe_mfma_raw(const uint16_t *A, const uint16_t *B,
                              const float *C, float *D, int ncase) {
  hipLaunchKernelGGL(raw_kernel, dim3(ncase), dim3(64), 0, 0, A, B, C, D,
                     ncase);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

extern "C" int probe_mfma_kstep(const float *XA, const float *XB, float *G,
                                int ncase) {
  hipLaunchKernelGGL(kstep_kernel, dim3(ncase), dim3(64), 0, 0, XA, XB, G,
                     ncase);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
