// VALU probe 3 (tools only, not shipped): issue cost of the INTEGER and
// compare/select instructions the order-statistic kernels are made of
// (v_min_u32, v_cndmask, v_sub_co/v_addc, v_bfe, v_lshl_or, v_mad_i32_i24,
// v_cmp, v_bitop3), against v_fmac_f32, at 1-4 waves per SIMD: SIMD-cycles
// per wave-instruction from the kernel time (clock from hipDeviceProp) and
// the ratio to v_fmac_f32 at the same occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIter = 4096;

#define OP2(ins, d, a) asm volatile(ins " %0, %0, %1" : "+v"(d) : "v"(a))

template <int MODE>
__global__ __launch_bounds__(256) void probe(unsigned *out) {
  unsigned s[16], t[16];
  double d[8], e[8];
  __shared__ unsigned lds[256 * 4];
  const unsigned lds_a = unsigned(uintptr_t(&lds[threadIdx.x])) & 0xFFFFu;
  unsigned long long mask = ~0ull >> (blockIdx.x & 7);
  asm volatile("" : "+s"(mask));
  for (int i = 0; i < 8; ++i) { d[i] = i * 0.5; e[i] = threadIdx.x * 1e-3; }
  for (int i = 0; i < 16; ++i) {
    s[i] = threadIdx.x * 3u + i;
    t[i] = threadIdx.x ^ (i * 77u);
  }
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (MODE == 0) OP2("v_fmac_f32", s[i], t[i]);
      if (MODE == 1) OP2("v_min_u32", s[i], t[i]);
      if (MODE == 2) OP2("v_add_u32", s[i], t[i]);
      if (MODE == 3) OP2("v_max_f32", s[i], t[i]);
      if (MODE == 4)
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 5)
        asm volatile("v_bfe_u32 %0, %0, 20, 11" : "+v"(s[i]));
      if (MODE == 6)
        asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 7)
        asm volatile("v_mad_i32_i24 %0, %0, %1, %0" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 8)
        asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(s[i]), "v"(t[i]) : "vcc");
      if (MODE == 9)
        asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x36" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 10)  // borrow into a counter: sub_co + addc (2 instr)
        asm volatile("v_sub_co_u32 %1, vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc"
                     : "+v"(s[i]), "+v"(t[i]) : "v"(s[(i + 1) & 15]) : "vcc");
      if (MODE == 11)
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 12)
        asm volatile("v_med3_f32 %0, %0, %1, %0" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 13)
        asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 14)
        asm volatile("v_min3_u32 %0, %0, %1, %0" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 15)
        asm volatile("v_cmp_gt_f32 vcc, %0, %1" :: "v"(s[i]), "v"(t[i]) : "vcc");
      if (MODE == 16)  // select on a mask held in an SGPR pair
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2"
                     : "+v"(s[i]) : "v"(t[i]), "s"(mask));
      if (MODE == 17)  // compare into vcc, then the select reading it
        asm volatile("v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc"
                     : "+v"(s[i]) : "v"(t[i]) : "vcc");
      if (MODE == 18)
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 19)
        asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 20)
        asm volatile("v_sub_u32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 21)
        asm volatile("v_max_u32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 22)  // 64-bit add of a double pair
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i & 7]) : "v"(e[i & 7]));
      if (MODE == 23)
        asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[i & 7]) : "v"(s[i]));
      if (MODE == 24)  // LDS atomic add (no return), per-lane word
        asm volatile("ds_add_u32 %0, %1" :: "v"(lds_a), "v"(t[i]));
      if (MODE == 25)
        asm volatile("ds_write_b32 %0, %1" :: "v"(lds_a), "v"(t[i]));
      if (MODE == 26)  // v_sub_co_u32 alone (borrow to vcc)
        asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(s[i]) : "v"(t[i]) : "vcc");
      if (MODE == 27)
        asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 28)
        asm volatile("v_min_i32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
      if (MODE == 29)
        asm volatile("v_min_f32 %0, %0, %1" : "+v"(s[i]) : "v"(t[i]));
    }
  }
  unsigned r = 0;
  for (int i = 0; i < 16; ++i) r += s[i] + t[i];
  for (int i = 0; i < 8; ++i) r += unsigned(d[i]);
  r += lds[threadIdx.x];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char *kName[] = {
    "v_fmac_f32", "v_min_u32", "v_add_u32", "v_max_f32", "v_cndmask_b32 vcc",
    "v_bfe_u32", "v_lshl_or_b32", "v_mad_i32_i24", "v_cmp_lt_u32 vcc",
    "v_bitop3_b32", "v_sub_co+v_addc (per instr)", "v_add_f32", "v_med3_f32",
    "v_pk_min_u16", "v_min3_u32", "v_cmp_gt_f32 vcc",
    "v_cndmask_b32_e64 sgpr-pair", "v_cmp vcc + v_cndmask (per instr)",
    "v_and_b32", "v_lshlrev_b32", "v_sub_u32", "v_max_u32", "v_add_f64",
    "v_cvt_f64_f32", "ds_add_u32", "ds_write_b32", "v_sub_co_u32",
    "v_xad_u32", "v_min_i32", "v_min_f32"};

template <int MODE>
double run(int wps, double ghz) {
  const int cus = 256;
  const int nb = cus * wps;  // 256-thread blocks: 4 waves, one per SIMD
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
  const double instr = double(kIter) * 16 * (MODE == 10 || MODE == 17 ? 2 : 1);
  return ms * 1e-3 * ghz * 1e9 / (instr * wps);  // SIMD-cycles per instr
}

template <int MODE>
void row(double ghz, const double *base) {
  printf("%-28s", kName[MODE]);
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
  printf("clock %.3f GHz (SIMD-cycles per wave-instruction; x = vs "
         "v_fmac_f32)\n", ghz);
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
  row<9>(ghz, base);
  row<10>(ghz, base);
  row<11>(ghz, base);
  row<12>(ghz, base);
  row<13>(ghz, base);
  row<14>(ghz, base);
  row<15>(ghz, base);
  row<16>(ghz, base);
  row<17>(ghz, base);
  row<18>(ghz, base);
  row<19>(ghz, base);
  row<20>(ghz, base);
  row<21>(ghz, base);
  row<22>(ghz, base);
  row<23>(ghz, base);
  row<24>(ghz, base);
  row<25>(ghz, base);
  row<26>(ghz, base);
  row<27>(ghz, base);
  row<28>(ghz, base);
  row<29>(ghz, base);
  return 0;
}
