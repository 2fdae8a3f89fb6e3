// FedOpt server-optimizer epilogue on the aggregated bucket (gfx950).
//
// FedOptAggregator.aggregate (federatedscope/core/aggregators/
// fedopt_aggregator.py:26-44) forms the pseudo-gradient g = model - avg and
// takes one step of the torch.optim optimizer the config names
// (core/auxiliaries/optimizer_builder.py:53-56: SGD, Adam, AdamW, Adagrad,
// RMSprop) on the server model.  Here the step is one fused elementwise pass
// over the device buckets — param, FedAvg result and the optimizer state are
// each read once and param/state written once (SGD: 16 B/elem with
// momentum, Adam: 24 B/elem, +8 with amsgrad, Adagrad 20 B, RMSprop 20-36) —
// following the arithmetic of torch's single-tensor CPU kernels (the
// reference runs the optimizer on CPU tensors): `add(alpha)` is a fused
// multiply-add (Vectorized fmadd), `lerp` with weight < 0.5 is
// self + w·(end − self) as an fma, `addcmul`/`addcdiv` are
// self + (v·t1)·t2 and self + (v·t1)/t2.  float32 and float64 parameters
// (the Python scalars enter as the tensor's type, as ATen casts them).
#include "common.h"

namespace fsagg {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float fma_t(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}
__device__ __forceinline__ double fma_t(double a, double b, double c) {
  return __builtin_fma(a, b, c);
}
// single-rounded ops of either type, never contracted
__device__ __forceinline__ float mul_t(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ double mul_t(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ float add_t(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ double add_t(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ float sub_t(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ double sub_t(double a, double b) { return __dsub_rn(a, b); }
__device__ __forceinline__ float div_t(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double div_t(double a, double b) { return __ddiv_rn(a, b); }
__device__ __forceinline__ float sqrt_t(float a) { return __fsqrt_rn(a); }
__device__ __forceinline__ double sqrt_t(double a) { return __dsqrt_rn(a); }

// the pseudo-gradient: model - new_model (fedopt_aggregator.py:35), negated
// for maximize (torch.optim: grad if not maximize else -grad)
template <typename T>
__device__ __forceinline__ T pseudo_grad(T x, T a, int flags) {
  const T g = sub_t(x, a);
  return (flags & FSAGG_OPT_MAXIMIZE) ? -g : g;
}

// torch.lerp(self, end, w) on CPU: self + w·(end − self) (an fma) for
// |w| < 0.5, end − (end − self)·(1 − w) otherwise
template <typename T>
__device__ __forceinline__ T lerp_t(T self, T end, T w) {
  return (w < T(0.5)) ? fma_t(w, sub_t(end, self), self)
                      : sub_t(end, mul_t(sub_t(end, self), sub_t(T(1), w)));
}

template <typename T>
__global__ __launch_bounds__(kBlock) void sgd_step_kernel(
    T *__restrict__ param, const T *__restrict__ avg, T *__restrict__ buf,
    int64_t numel, fsagg_opt_params hp) {
  const bool nesterov = hp.flags & FSAGG_OPT_NESTEROV;
  const bool first = hp.flags & FSAGG_OPT_FIRST_STEP;
  const T lr = T(hp.lr), wd = T(hp.weight_decay), mom = T(hp.momentum);
  const T keep = T(1.0 - hp.dampening);  // Python's 1 - dampening
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const T x = param[p];
    T g = pseudo_grad(x, avg[p], hp.flags);
    if (hp.weight_decay != 0.0) g = fma_t(x, wd, g);
    if (hp.momentum != 0.0) {
      T b;
      if (first) {
        b = g;  // torch.clone(grad)
      } else {
        b = mul_t(buf[p], mom);
        b = fma_t(g, keep, b);
      }
      buf[p] = b;
      g = nesterov ? fma_t(b, mom, g) : b;
    }
    param[p] = fma_t(g, -lr, x);
  }
}

template <typename T, bool AMS>
__global__ __launch_bounds__(kBlock) void adam_step_kernel(
    T *__restrict__ param, const T *__restrict__ avg, T *__restrict__ m1,
    T *__restrict__ m2, T *__restrict__ vmax, int64_t numel,
    fsagg_opt_params hp) {
  const T w1 = T(1.0 - hp.beta1);  // lerp weight, Python's 1 - beta1
  const T w2 = T(1.0 - hp.beta2);  // addcmul value
  const T b2 = T(hp.beta2), wd = T(hp.weight_decay), eps = T(hp.eps);
  const T bc2 = T(hp.bias_correction2_sqrt), neg_step = T(-hp.step_size);
  const bool decoupled = hp.flags & FSAGG_OPT_DECOUPLED;
  const T dmul = T(hp.decay_mul);  // AdamW: param.mul_(1 - lr * wd)
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    T x = param[p];
    T g = pseudo_grad(x, avg[p], hp.flags);
    if (hp.weight_decay != 0.0) {
      if (decoupled) x = mul_t(x, dmul);
      else g = fma_t(x, wd, g);
    }
    // exp_avg.lerp_(grad, 1 - beta1)
    const T a = lerp_t(m1[p], g, w1);
    T v = mul_t(m2[p], b2);
    v = add_t(v, mul_t(mul_t(w2, g), g));  // addcmul_(g, g, 1 - beta2)
    m1[p] = a;
    m2[p] = v;
    T vd = v;
    if (AMS) {  // torch.maximum(max_exp_avg_sq, exp_avg_sq, out=...)
      const T mx = vmax[p];
      vd = (mx != mx || v != v) ? (mx != mx ? mx : v) : (mx > v ? mx : v);
      vmax[p] = vd;
    }
    const T denom = add_t(div_t(sqrt_t(vd), bc2), eps);
    // param.addcdiv_(exp_avg, denom, value=-step_size)
    param[p] = add_t(x, div_t(mul_t(neg_step, a), denom));
  }
}

// torch.optim Adagrad (_single_tensor_adagrad): state_sum.addcmul_(g, g,
// value=1); std = sqrt(state_sum) + eps; param.addcdiv_(g, std,
// value=-clr)
template <typename T>
__global__ __launch_bounds__(kBlock) void adagrad_step_kernel(
    T *__restrict__ param, const T *__restrict__ avg, T *__restrict__ sum,
    int64_t numel, fsagg_opt_params hp) {
  const T wd = T(hp.weight_decay), eps = T(hp.eps), neg_clr = T(-hp.clr);
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const T x = param[p];
    T g = pseudo_grad(x, avg[p], hp.flags);
    if (hp.weight_decay != 0.0) g = fma_t(x, wd, g);
    const T ss = add_t(sum[p], mul_t(g, g));  // (1·g)·g
    sum[p] = ss;
    const T sd = add_t(sqrt_t(ss), eps);
    param[p] = add_t(x, div_t(mul_t(neg_clr, g), sd));
  }
}

// torch.optim RMSprop (_single_tensor_rmsprop): square_avg.mul_(alpha)
// .addcmul_(g, g, value=1-alpha); centered: grad_avg.lerp_(g, 1-alpha),
// avg = sqrt(square_avg.addcmul(grad_avg, grad_avg, value=-1)); else
// avg = sqrt(square_avg); avg += eps; momentum: buf.mul_(momentum)
// .addcdiv_(g, avg), param.add_(buf, alpha=-lr); else param.addcdiv_(g,
// avg, value=-lr)
template <typename T, bool CENTERED, bool MOM>
__global__ __launch_bounds__(kBlock) void rmsprop_step_kernel(
    T *__restrict__ param, const T *__restrict__ avg, T *__restrict__ sq,
    T *__restrict__ buf, T *__restrict__ gavg, int64_t numel,
    fsagg_opt_params hp) {
  const T wd = T(hp.weight_decay), eps = T(hp.eps), alpha = T(hp.alpha);
  const T w = T(1.0 - hp.alpha), mom = T(hp.momentum), neg_lr = T(-hp.lr);
  for (int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x; p < numel;
       p += int64_t(gridDim.x) * kBlock) {
    const T x = param[p];
    T g = pseudo_grad(x, avg[p], hp.flags);
    if (hp.weight_decay != 0.0) g = fma_t(x, wd, g);
    T v = mul_t(sq[p], alpha);
    v = add_t(v, mul_t(mul_t(w, g), g));
    sq[p] = v;
    T d;
    if (CENTERED) {
      const T ga = lerp_t(gavg[p], g, w);
      gavg[p] = ga;
      d = sqrt_t(add_t(v, mul_t(mul_t(T(-1), ga), ga)));
    } else {
      d = sqrt_t(v);
    }
    d = add_t(d, eps);
    if (MOM) {
      T b = mul_t(buf[p], mom);
      b = add_t(b, div_t(g, d));  // addcdiv value 1: (1·g)/avg
      buf[p] = b;
      param[p] = fma_t(b, neg_lr, x);
    } else {
      param[p] = add_t(x, div_t(mul_t(neg_lr, g), d));
    }
  }
}

template <typename T>
int opt_step(T *param, const T *avg, T *state0, T *state1, T *state2,
             int64_t numel, const fsagg_opt_params *hp, fsagg_stream_t stream,
             const char *what) {
  if (!param || !avg || !hp || numel < 0) {
    set_error("%s: invalid argument", what);
    return FSAGG_EINVAL;
  }
  if (numel == 0) return FSAGG_OK;
  const unsigned grid = stream_grid(numel, kBlock, 256 * 8);
  hipStream_t s = as_stream(stream);
  switch (hp->kind) {
    case FSAGG_OPT_SGD:
      if (hp->momentum != 0.0 && !state0) {
        set_error("%s: SGD momentum needs state0", what);
        return FSAGG_EINVAL;
      }
      hipLaunchKernelGGL(sgd_step_kernel<T>, dim3(grid), dim3(kBlock), 0, s,
                         param, avg, state0, numel, *hp);
      break;
    case FSAGG_OPT_ADAM:
      if (!state0 || !state1 || ((hp->flags & FSAGG_OPT_AMSGRAD) && !state2)) {
        set_error("%s: Adam needs state0 and state1 (and state2 with "
                  "amsgrad)", what);
        return FSAGG_EINVAL;
      }
      if (hp->flags & FSAGG_OPT_AMSGRAD)
        hipLaunchKernelGGL((adam_step_kernel<T, true>), dim3(grid),
                           dim3(kBlock), 0, s, param, avg, state0, state1,
                           state2, numel, *hp);
      else
        hipLaunchKernelGGL((adam_step_kernel<T, false>), dim3(grid),
                           dim3(kBlock), 0, s, param, avg, state0, state1,
                           state2, numel, *hp);
      break;
    case FSAGG_OPT_ADAGRAD:
      if (!state0) {
        set_error("%s: Adagrad needs state0", what);
        return FSAGG_EINVAL;
      }
      hipLaunchKernelGGL(adagrad_step_kernel<T>, dim3(grid), dim3(kBlock), 0,
                         s, param, avg, state0, numel, *hp);
      break;
    case FSAGG_OPT_RMSPROP: {
      const bool centered = hp->flags & FSAGG_OPT_CENTERED;
      const bool mom = hp->momentum > 0.0;
      if (!state0 || (mom && !state1) || (centered && !state2)) {
        set_error("%s: RMSprop needs state0 (and state1 with momentum, "
                  "state2 when centered)", what);
        return FSAGG_EINVAL;
      }
#define FSAGG_RMS(C, M)                                                      \
  hipLaunchKernelGGL((rmsprop_step_kernel<T, C, M>), dim3(grid), dim3(kBlock), \
                     0, s, param, avg, state0, state1, state2, numel, *hp)
      if (centered) {
        if (mom) FSAGG_RMS(true, true); else FSAGG_RMS(true, false);
      } else {
        if (mom) FSAGG_RMS(false, true); else FSAGG_RMS(false, false);
      }
#undef FSAGG_RMS
      break;
    }
    default:
      set_error("%s: unknown optimizer kind %d", what, hp->kind);
      return FSAGG_EINVAL;
  }
  return check_launch(what);
}

}  // namespace
}  // namespace fsagg

using namespace fsagg;

extern "C" int fsagg_server_opt_step_f32(float *param, const float *avg,
                                         float *state0, float *state1,
                                         float *state2, int64_t numel,
                                         const fsagg_opt_params *hp,
                                         fsagg_stream_t stream) {
  return opt_step<float>(param, avg, state0, state1, state2, numel, hp,
                         stream, "fsagg_server_opt_step_f32");
}

extern "C" int fsagg_server_opt_step_f64(double *param, const double *avg,
                                         double *state0, double *state1,
                                         double *state2, int64_t numel,
                                         const fsagg_opt_params *hp,
                                         fsagg_stream_t stream) {
  return opt_step<double>(param, avg, state0, state1, state2, numel, hp,
                          stream, "fsagg_server_opt_step_f64");
}
