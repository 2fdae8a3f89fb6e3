// FedOpt server-optimizer epilogue on the aggregated bucket (gfx950).
//
// FedOptAggregator.aggregate (federatedscope/core/aggregators/
// fedopt_aggregator.py:26-44) forms the pseudo-gradient g = model - avg and
// takes one torch.optim step on the server model.  Here the step is one
// fused elementwise pass over the device buckets — param, FedAvg result and
// the optimizer state are each read once and param/state written once
// (SGD: 16 B/elem with momentum, Adam: 24 B/elem) — following the
// arithmetic of torch's single-tensor CPU kernels (the reference runs the
// optimizer on CPU tensors): `add(alpha)` is a fused multiply-add
// (Vectorized fmadd), `lerp` with weight < 0.5 is self + w·(end − self) as an
// fma, `addcmul`/`addcdiv` are self + (v·t1)·t2 and self + (v·t1)/t2.
#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float fma_rn(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}

__global__ __launch_bounds__(kBlock) void sgd_step_kernel(
    float *__restrict__ param, const float *__restrict__ avg,
    float *__restrict__ buf, int64_t numel, fsagg_opt_params hp) {
  const bool nesterov = hp.flags & FSAGG_OPT_NESTEROV;
  const bool first = hp.flags & FSAGG_OPT_FIRST_STEP;
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const float x = param[p];
    float g = x - avg[p];  // grads = model - new_model  (fedopt_aggregator.py:35)
    if (hp.weight_decay != 0.0f) g = fma_rn(x, hp.weight_decay, g);
    if (hp.momentum != 0.0f) {
      float b;
      if (first) {
        b = g;  // torch.clone(grad)
      } else {
        b = mul_rn(buf[p], hp.momentum);
        b = fma_rn(g, 1.0f - hp.dampening, b);
      }
      buf[p] = b;
      g = nesterov ? fma_rn(b, hp.momentum, g) : b;
    }
    param[p] = fma_rn(g, -hp.lr, x);
  }
}

__global__ __launch_bounds__(kBlock) void adam_step_kernel(
    float *__restrict__ param, const float *__restrict__ avg,
    float *__restrict__ m1, float *__restrict__ m2, int64_t numel,
    fsagg_opt_params hp) {
  const float w1 = 1.0f - hp.beta1;
  const float w2 = 1.0f - hp.beta2;
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const float x = param[p];
    float g = x - avg[p];
    if (hp.weight_decay != 0.0f) g = fma_rn(x, hp.weight_decay, g);
    float a = m1[p];
    // exp_avg.lerp_(grad, 1 - beta1)
    a = (w1 < 0.5f) ? fma_rn(w1, g - a, a) : g - mul_rn(g - a, 1.0f - w1);
    float v = mul_rn(m2[p], hp.beta2);
    v = add_rn(v, mul_rn(mul_rn(w2, g), g));      // addcmul_(g, g, 1 - beta2)
    const float denom =
        add_rn(__fdiv_rn(__fsqrt_rn(v), hp.bias_correction2_sqrt), hp.eps);
    m1[p] = a;
    m2[p] = v;
    // param.addcdiv_(exp_avg, denom, value=-step_size)
    param[p] = add_rn(x, __fdiv_rn(mul_rn(-hp.step_size, a), denom));
  }
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_server_opt_step_f32(float *param, const float *avg,
                                         float *state0, float *state1,
                                         int64_t numel,
                                         const fsagg_opt_params *hp,
                                         fsagg_stream_t stream) {
  if (!param || !avg || !hp || numel < 0) {
    set_error("fsagg_server_opt_step_f32: invalid argument");
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  const unsigned grid = stream_grid(numel, kBlock, 256 * 8);
  hipStream_t s = as_stream(stream);
  switch (hp->kind) {
    case FSAGG_OPT_SGD:
      if (hp->momentum != 0.0f && !state0) {
        set_error("fsagg_server_opt_step_f32: SGD momentum needs state0");
        return FSAGG_EINVAL;
      }
      hipLaunchKernelGGL(sgd_step_kernel, dim3(grid), dim3(kBlock), 0, s,
                         param, avg, state0, numel, *hp);
      break;
    case FSAGG_OPT_ADAM:
      if (!state0 || !state1) {
        set_error("fsagg_server_opt_step_f32: Adam needs state0 and state1");
        return FSAGG_EINVAL;
      }
      hipLaunchKernelGGL(adam_step_kernel, dim3(grid), dim3(kBlock), 0, s,
                         param, avg, state0, state1, numel, *hp);
      break;
    default:
      set_error("fsagg_server_opt_step_f32: unknown optimizer kind %d",
                hp->kind);
      return FSAGG_EINVAL;
  }
  return check_launch("fsagg_server_opt_step_f32");
}
