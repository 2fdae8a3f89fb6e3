// VALU probe 4 (tools only, not shipped): issue cost of the fp64 and
// broadcast instructions the selected-rows distance kernel (pairsel.hip)
// is made of — v_fma_f64, v_add_f64 (VGPR and SGPR-pair operands),
// v_readlane_b32, ds_read_b128 / ds_read_b64 with one address for the whole
// wave (broadcast), ds_read_b32 with 64 distinct addresses — at 1-4 waves
// per SIMD: SIMD-cycles per wave-instruction (clock from hipDeviceProp),
// and the ratio to v_fmac_f32.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIter = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void probe(unsigned *out) {
  unsigned s[16], t[16];
  double d[8], e[8];
  __shared__ __attribute__((aligned(16))) unsigned lds[256 * 4];
  const unsigned lds_a = unsigned(uintptr_t(&lds[threadIdx.x])) & 0xFFFFu;
  const unsigned lds_0 = unsigned(uintptr_t(&lds[0])) & 0xFFFFu;
  unsigned long long sd = 0x3FD0000000000000ull + (blockIdx.x & 7);
  asm volatile("" : "+s"(sd));
  for (int i = 0; i < 8; ++i) { d[i] = i * 0.5; e[i] = threadIdx.x * 1e-3; }
  for (int i = 0; i < 16; ++i) {
    s[i] = threadIdx.x * 3u + i;
    t[i] = threadIdx.x ^ (i * 77u);
  }
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  unsigned sg = 0;
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (MODE == 0)
        asm volatile("v_fmac_f32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 1)
        asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(d[i & 7]) : "v"(e[i & 7]));
      if (MODE == 2)
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i & 7]) : "v"(e[i & 7]));
      if (MODE == 3)
        asm volatile("v_add_f64 %0, %1, -%0" : "+v"(d[i & 7]) : "s"(sd));
      if (MODE == 4) {
        asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(sg) : "v"(s[i]), "n"(5));
        asm volatile("" :: "s"(sg));
      }
      if (MODE == 5) {
        unsigned a, b, c, dd;
        asm volatile("ds_read_b128 %0, %1" : "=v"(*(__attribute__((ext_vector_type(4))) unsigned *)&s[i & 12]) : "v"(lds_0));
        (void)a; (void)b; (void)c; (void)dd;
      }
      if (MODE == 6)
        asm volatile("ds_read_b64 %0, %1" : "=v"(d[i & 7]) : "v"(lds_0));
      if (MODE == 7)
        asm volatile("ds_read_b32 %0, %1" : "=v"(s[i]) : "v"(lds_a));
      if (MODE == 8)
        asm volatile("ds_read_b128 %0, %1" : "=v"(*(__attribute__((ext_vector_type(4))) unsigned *)&s[i & 12]) : "v"(lds_a * 4 & 0xFFF0u));
    }
    if (MODE >= 5) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  unsigned r = sg;
  for (int i = 0; i < 16; ++i) r += s[i] + t[i];
  for (int i = 0; i < 8; ++i) r += unsigned(d[i]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char *kName[] = {
    "v_fmac_f32", "v_fma_f64", "v_add_f64", "v_add_f64 sgpr-pair",
    "v_readlane_b32", "ds_read_b128 broadcast", "ds_read_b64 broadcast",
    "ds_read_b32 distinct", "ds_read_b128 distinct"};

template <int MODE>
double run(int wps, double ghz) {
  const int nb = 256 * wps;
  unsigned *out;
  hipMalloc(&out, sizeof(unsigned) * nb * 256);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), 0, 0, out);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(256), 0, 0, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipFree(out);
  return ms * 1e-3 * ghz * 1e9 / (double(kIter) * 16 * wps);
}

template <int MODE>
void row(double ghz, const double *base) {
  printf("%-26s", kName[MODE]);
  for (int w = 1; w <= 4; ++w) {
    const double c = run<MODE>(w, ghz);
    printf("  w%d %.2f (x%.2f)", w, c, c / base[w - 1]);
  }
  printf("\n");
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const double ghz = p.clockRate / 1e6;
  printf("clock %.3f GHz (SIMD-cycles per wave-instruction)\n", ghz);
  double base[4];
  for (int w = 1; w <= 4; ++w) base[w - 1] = run<0>(w, ghz);
  row<0>(ghz, base);
  row<1>(ghz, base);
  row<2>(ghz, base);
  row<3>(ghz, base);
  row<4>(ghz, base);
  row<5>(ghz, base);
  row<6>(ghz, base);
  row<7>(ghz, base);
  row<8>(ghz, base);
  return 0;
}
