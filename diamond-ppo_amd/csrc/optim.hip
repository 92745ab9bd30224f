// Gradient slab reduction, clip_grad_norm_ and Adam on gfx950.
//
// Replaces, per minibatch, loss.backward()'s parameter-gradient accumulation (ppo.py:283),
// nn.utils.clip_grad_norm_(params, 0.5) (ppo.py:284; torch nn/utils/clip_grad.py:96,106,165,169)
// and optimizer.step() (ppo.py:285; torch optim/adam.py _single_tensor_adam, the CPU path the
// reference runs: step += 1; exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
// denom = sqrt(exp_avg_sq)/sqrt(bc2) + eps; p.addcdiv_(exp_avg, denom, -lr/bc1)).
//
// Both kernels are HBM/L2-latency bound and tiny (P ~ 13-14 K floats): the slab reduction reads
// G slabs of P floats once (fixed order => bit-reproducible); every Adam workgroup recomputes the
// global norm from the reduced gradient (52 KB, L2-resident) so no grid-wide sync is needed.
#include "common.h"

namespace dppo {
namespace {

__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slabs, int G,
                                                          int64_t stride, int64_t p_total,
                                                          float* __restrict__ grad,
                                                          int64_t ls_off, int ls_n, float ent_coef,
                                                          int add_entropy_const) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= p_total + 8) return;
  float s = 0.0f;
  for (int g = 0; g < G; ++g) s += slabs[(int64_t)g * stride + p];
  // d(-beta * mean H)/d log_std = -beta per action dim (continuous_ppo.py:286-291): a constant
  // the per-sample kernel does not see; added once (rank 0 only under data parallelism).
  if (add_entropy_const && p >= ls_off && p < ls_off + ls_n) s -= ent_coef;
  grad[p] = s;
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sh[w];
  return t;
}

// grad: [n] flat gradient followed by 8 loss slots {sum l_pi, sum l_v, sum H, ...}.
__global__ __launch_bounds__(256) void clip_adam_kernel(
    float* __restrict__ params, float* __restrict__ grad, float* __restrict__ m,
    float* __restrict__ v, int64_t n, float max_norm, float lr, float neg_step_size,
    float bc2_sqrt, float beta1, float beta2, float eps, float* __restrict__ out_norm,
    float* __restrict__ trace, float inv_m, float vf, float ent) {
#pragma clang fp contract(off)
  __shared__ double sh[4];
  double sq = 0.0;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const double g = grad[k];
    sq += g * g;
  }
  const double tot = block_sum(sq, sh);
  const float norm = (float)sqrt(tot);
  // clip_coef = max_norm / (total_norm + 1e-6), clamped to 1, always applied (clip_grad.py:165-169)
  float coef = max_norm / (norm + 1e-6f);
  coef = coef < 1.0f ? coef : 1.0f;
  const float w1 = 1.0f - beta1;
  const float w2 = 1.0f - beta2;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const float g = grad[k] * coef;
    float mk = m[k];
    mk = mk + w1 * (g - mk);                 // lerp, weight < 0.5 branch
    float vk = v[k] * beta2;
    vk = vk + (w2 * g) * g;                  // addcmul_(g, g, value = 1 - beta2)
    const float denom = sqrtf(vk) / bc2_sqrt + eps;
    params[k] = params[k] + neg_step_size * (mk / denom);
    m[k] = mk;
    v[k] = vk;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (out_norm) *out_norm = norm;
    if (trace) {
      const float lpi = grad[n + 0] * inv_m;
      const float lv = grad[n + 1] * inv_m;
      const float h = grad[n + 2] * inv_m;
      trace[0] = lpi + vf * lv - ent * h;  // ppo.py:276-280
      trace[1] = lpi;
      trace[2] = lv;
      trace[3] = h;
      trace[4] = norm;
    }
  }
}

}  // namespace

int launch_slab_reduce(const float* slabs, int G, int64_t slab_stride, int64_t p_total,
                       float* grad, float* /*loss4*/, float /*inv_m*/, int64_t ls_off, int ls_n,
                       float ent_coef, int add_entropy_const, hipStream_t s) {
  const int64_t n = p_total + 8;
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid), dim3(256), 0, s, slabs, G, slab_stride,
                     p_total, grad, ls_off, ls_n, ent_coef, add_entropy_const);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_clip_adam_traced(float* params, float* grad, float* m, float* v, int64_t n,
                            float max_norm, float lr, float neg_step_size, float bc2_sqrt,
                            float beta1, float beta2, float eps, float* out_norm, float* trace,
                            float inv_m, float vf, float ent, hipStream_t s) {
  int64_t g = (n + 255) / 256;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(clip_adam_kernel, dim3((unsigned)g), dim3(256), 0, s, params, grad, m, v, n,
                     max_norm, lr, neg_step_size, bc2_sqrt, beta1, beta2, eps, out_norm, trace,
                     inv_m, vf, ent);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_clip_adam(float* params, float* grad, float* m, float* v, int64_t n, float max_norm,
                     float lr, float neg_step_size, float bc2_sqrt, float beta1, float beta2,
                     float eps, float* out_norm, hipStream_t s) {
  return launch_clip_adam_traced(params, grad, m, v, n, max_norm, lr, neg_step_size, bc2_sqrt,
                                 beta1, beta2, eps, out_norm, nullptr, 0.f, 0.f, 0.f, s);
}

}  // namespace dppo
