// The K-wave order-statistic kernel (orderstat_group.h) for 255 < n <= 512
// clients, one instantiation per per-wave register-array size.
#include "orderstat_group.h"

namespace fsagg {
namespace os {

template <int H, int MODE>
void launch_group_h(const RowSrc &rs, unsigned grid, int n, int kk,
                    float divisor, float *out, int waves, hipStream_t s) {
  hipLaunchKernelGGL((orderstat_group_kernel<H, MODE>), dim3(grid),
                     dim3(waves * kWave), 0, s, rs, n, kk, divisor, out);
}

std::atomic<int> g_group_waves{kGroupMaxWaves};

template <int MODE>
bool launch_group(const RowSrc &rs, unsigned grid, int n, int kk,
                  float divisor, float *out, hipStream_t s) {
  // eight waves per block whatever n: two blocks (the LDS they take) fill a
  // CU's 16 wave slots — five waves per block at n = 300 left 10 of 16 and
  // ran slower than the two-pass streaming kernel
  // (fsagg_orderstat_set_group_waves moves it for A/B)
  const int K = g_group_waves.load(std::memory_order_relaxed);
  if (n <= 64 || n > K * kGroupRows) return false;
  const int per = (n + K - 1) / K;
  switch ((per + 7) / 8 * 8) {
    case 32: launch_group_h<32, MODE>(rs, grid, n, kk, divisor, out, K, s); break;
    case 40: launch_group_h<40, MODE>(rs, grid, n, kk, divisor, out, K, s); break;
    case 48: launch_group_h<48, MODE>(rs, grid, n, kk, divisor, out, K, s); break;
    case 56: launch_group_h<56, MODE>(rs, grid, n, kk, divisor, out, K, s); break;
    case 64: launch_group_h<64, MODE>(rs, grid, n, kk, divisor, out, K, s); break;
    default: return false;
  }
  return true;
}

template bool launch_group<kMedian>(const RowSrc &, unsigned, int, int, float,
                                    float *, hipStream_t);
template bool launch_group<kTrimmed>(const RowSrc &, unsigned, int, int, float,
                                     float *, hipStream_t);

}  // namespace os
}  // namespace fsagg
