// VALU probe 2 (tools only): the Krum inner-loop pattern — packed
// (x_pair − broadcast y)² accumulate — with and without operand modifiers,
// at 2 waves per SIMD; cycles per packed instruction per SIMD from the
// kernel time at an assumed 2.1 GHz plus the per-wave s_memtime count.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 8192;

// d = x − {y.lo, y.lo}: op_sel_hi:[1,0] takes y's low half for the high
// lane; neg on src1 turns the add into a subtraction
#define PK_SUB_BC(d, x, y) asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(x), "v"(y))
#define PK_ADD(d, x, y) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(d) : "v"(x), "v"(y))
#define PK_SQACC(a, d) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(a) : "v"(d))

template <int MODE>
__global__ __launch_bounds__(256) void probe(float *out, long long *cyc) {
  f2 acc[10], x[5], y[5];
  for (int i = 0; i < 10; ++i) acc[i] = f2{0.f, 0.f};
  for (int i = 0; i < 5; ++i) { x[i] = f2{threadIdx.x * 1e-9f, i * 1e-9f}; y[i] = f2{i * 1e-7f, 1e-8f}; }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int v = 0; v < 10; v += 2) {
      f2 d0, d1;
      if (MODE == 0) {  // broadcast + neg modifiers, 2 temps interleaved
        PK_SUB_BC(d0, x[v / 2], y[v / 2]);
        PK_SUB_BC(d1, x[(v / 2 + 1) % 5], y[v / 2]);
      } else {          // plain
        PK_ADD(d0, x[v / 2], y[v / 2]);
        PK_ADD(d1, x[(v / 2 + 1) % 5], y[v / 2]);
      }
      PK_SQACC(acc[v], d0);
      PK_SQACC(acc[v + 1], d1);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int i = 0; i < 10; ++i) r += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name) {
  for (int wps : {1, 2}) {
    const int nb = 256 * wps;  // 256-thread blocks: one wave per SIMD each
    float *out; long long *cyc;
    (void)hipMalloc(&out, sizeof(float) * nb * 256);
    (void)hipMalloc(&cyc, sizeof(long long) * nb * 4);
    hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), 0, 0, out, cyc);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), 0, 0, out, cyc);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    long long *h = new long long[nb * 4];
    (void)hipMemcpy(h, cyc, sizeof(long long) * nb * 4, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < nb * 4; ++i) avg += h[i]; avg /= nb * 4;
    const double per_wave = double(kIter) * 20;  // 10 sub + 10 fma
    printf("%-22s waves/SIMD=%d ms=%.4f ticks/instr/wave=%.3f cyc/instr/SIMD@2.1GHz=%.3f\n",
           name, wps, ms, avg / per_wave, ms * 1e-3 * 2.1e9 / (per_wave * wps));
    delete[] h; (void)hipFree(out); (void)hipFree(cyc);
  }
}

int main() {
  run<0>("bcast+neg modifiers");
  run<1>("plain");
  return 0;
}
