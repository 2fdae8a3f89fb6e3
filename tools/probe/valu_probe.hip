// VALU issue-model probe for gfx950 (tools only, not shipped): cycles per
// instruction, per wave (s_memtime), for packed/scalar f32 FMA streams at 1,
// 2 and 4 waves per SIMD, independent and dependent forms.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 4096;

#define PK_FMA(a, b) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(a) : "v"(b))
#define PK_ADD(d, a, b) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))
#define FMA(a, b) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(a) : "v"(b))
#define SUB(d, a, b) asm volatile("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b))

template <int MODE>
__global__ __launch_bounds__(256) void probe(float *out, long long *cyc) {
  f2 acc[8], x[8];
  float s[16], t[16];
  for (int i = 0; i < 8; ++i) { acc[i] = f2{0.f, 0.f}; x[i] = f2{threadIdx.x * 1e-9f, i * 1e-9f}; }
  for (int i = 0; i < 16; ++i) { s[i] = 0.f; t[i] = threadIdx.x * 1e-9f + i; }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIter; ++it) {
    if (MODE == 0) {  // 8 independent pk_fma
#pragma unroll
      for (int i = 0; i < 8; ++i) PK_FMA(acc[i], x[i]);
    } else if (MODE == 1) {  // 16 independent v_fmac
#pragma unroll
      for (int i = 0; i < 16; ++i) FMA(s[i], t[i]);
    } else if (MODE == 2) {  // pk_add then its dependent pk_fma, back to back
#pragma unroll
      for (int i = 0; i < 8; ++i) { f2 d; PK_ADD(d, x[i], acc[(i + 1) & 7]); PK_FMA(acc[i], d); }
    } else if (MODE == 3) {  // 4 pk_add, then the 4 dependent pk_fma
#pragma unroll
      for (int h = 0; h < 8; h += 4) {
        f2 d0, d1, d2, d3;
        PK_ADD(d0, x[h], x[h + 4]); PK_ADD(d1, x[h + 1], x[h + 5]);
        PK_ADD(d2, x[h + 2], x[h + 6]); PK_ADD(d3, x[h + 3], x[h + 7]);
        PK_FMA(acc[h], d0); PK_FMA(acc[h + 1], d1); PK_FMA(acc[h + 2], d2); PK_FMA(acc[h + 3], d3);
      }
    } else if (MODE == 4) {  // scalar sub then dependent fma, back to back
#pragma unroll
      for (int i = 0; i < 16; ++i) { float d; SUB(d, t[i], t[(i + 1) & 15]); FMA(s[i], d); }
    } else if (MODE == 5) {  // scalar: 4 subs then 4 fmas
#pragma unroll
      for (int h = 0; h < 16; h += 4) {
        float d0, d1, d2, d3;
        SUB(d0, t[h], t[h ^ 8]); SUB(d1, t[h + 1], t[(h + 1) ^ 8]);
        SUB(d2, t[h + 2], t[(h + 2) ^ 8]); SUB(d3, t[h + 3], t[(h + 3) ^ 8]);
        FMA(s[h], d0); FMA(s[h + 1], d1); FMA(s[h + 2], d2); FMA(s[h + 3], d3);
      }
    } else if (MODE == 6) {  // one pk_fma chain (dependent)
#pragma unroll
      for (int i = 0; i < 8; ++i) PK_FMA(acc[0], x[i]);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int i = 0; i < 8; ++i) r += acc[i].x + acc[i].y;
  for (int i = 0; i < 16; ++i) r += s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int per_iter) {
  int cus = 256;
  for (int wps : {1, 2, 4}) {
    const int blocks = cus, threads = 64 * 4 * wps;  // 4 SIMDs × wps waves
    float *out; long long *cyc;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads > 256 ? 256 : threads), 0, 0, out, cyc);
    hipDeviceSynchronize();
    // (256-thread blocks: launch enough of them for wps waves per SIMD)
    const int nb = blocks * threads / 256;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), 0, 0, out, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const int nw = nb * 4;
    long long *h = new long long[nw];
    hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < nw; ++i) avg += h[i]; avg /= nw;
    const double instr = double(kIter) * per_iter;
    // memtime ticks at 100 MHz on some parts: report both forms
    printf("%-28s waves/SIMD=%d  ms=%.4f  ticks/wave=%.0f  ticks/instr/wave=%.3f  "
           "SIMD-cycles/instr @2.1GHz=%.3f\n", name, wps, ms, avg, avg / instr,
           ms * 1e-3 * 2.1e9 / (instr * wps));
    delete[] h; hipFree(out); hipFree(cyc);
  }
}

int main() {
  run<0>("pk_fma x8 indep", 8);
  run<1>("v_fmac x16 indep", 16);
  run<2>("pk_add->pk_fma b2b", 16);
  run<3>("4 pk_add, 4 pk_fma", 16);
  run<4>("sub->fmac b2b", 32);
  run<5>("4 sub, 4 fmac", 32);
  run<6>("pk_fma one chain", 8);
  return 0;
}
