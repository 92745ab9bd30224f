// GAE, advantage statistics / normalisation, and sample-record packing for gfx950.
//
// GAE replaces PPO.calculate_advantage (reference diamond/ppo.py:188-222; identical code in
// continuous_ppo.py:200-234 and recurrent_ppo.py:265-299) fused with returns = values + adv
// (ppo.py:241) and the per-tile partial sums for the normalisation (ppo.py:243).
//
// Roofline: HBM-bound, 22 algorithmic bytes per element (rewards, values, next_values 4 B each,
// term/trunc 1 B each read; advantages and returns 4 B each written), ~0.5 FLOP/B.
//
// Mapping: one workgroup (256 threads) owns a tile of kEnvTile envs x a chunk of T steps.  All
// 256 threads stage the chunk's rows into LDS with 16-byte loads (each row is contiguous along
// the env axis), then one lane per env runs the serial backward recurrence out of LDS in the
// reference's exact fp32 operation order, and all threads write adv/returns back with 16-byte
// stores.  The recurrence is serial per env (bit-exactness forbids re-association), but it is
// only 2 dependent flops per step; the bytes are what cost, and they move with every lane of
// the chip busy: N/kEnvTile workgroups (512 at N = 8192, several per CU so one tile's scan
// overlaps the next tile's loads).
#include "common.h"

namespace dppo {
namespace {

constexpr int kEnvTile = 16;   // envs per workgroup: 64-B f32 rows, 16-B flag rows
constexpr int kTChunk = 128;   // steps staged per pass (28 KiB of LDS)
constexpr int kThreads = 256;

// The reference op order, with FMA contraction disabled:
//   nt = 1 - term; ntr = 1 - trunc                                    (ppo.py:202-203)
//   delta = (r + (gamma * nv) * nt) - v                               (ppo.py:206-210)
//   a = delta + ((c * nt) * ntr) * a,  c = fp32(gamma * lambda in double)   (ppo.py:213-220)
__device__ __forceinline__ float gae_step(float a, float r, float v, float nv, float te, float tr,
                                          float g, float c) {
#pragma clang fp contract(off)
  const float nt = 1.0f - te;
  const float ntr = 1.0f - tr;
  const float delta = (r + (g * nv) * nt) - v;
  return delta + ((c * nt) * ntr) * a;
}

template <bool kVec>
__global__ __launch_bounds__(kThreads) void gae_kernel(
    const float* __restrict__ rew, const uint8_t* __restrict__ term,
    const uint8_t* __restrict__ trunc, const float* __restrict__ val,
    const float* __restrict__ nval, float* __restrict__ adv, float* __restrict__ ret,
    double* __restrict__ partials, int T, int N, float g, float c) {
  __shared__ __attribute__((aligned(16))) float s_r[kTChunk][kEnvTile];
  __shared__ __attribute__((aligned(16))) float s_v[kTChunk][kEnvTile];
  __shared__ __attribute__((aligned(16))) float s_nv[kTChunk][kEnvTile];
  __shared__ __attribute__((aligned(16))) uint8_t s_te[kTChunk][kEnvTile];
  __shared__ __attribute__((aligned(16))) uint8_t s_tr[kTChunk][kEnvTile];

  const int tid = threadIdx.x;
  const int n0 = blockIdx.x * kEnvTile;
  const int my_n = n0 + tid;  // scan lane (tid < kEnvTile)
  float a = 0.0f;             // advantage carried backwards (ppo.py:198)
  double sum = 0.0, sumsq = 0.0;

  for (int t_hi = T; t_hi > 0; t_hi -= kTChunk) {
    const int t_lo = t_hi > kTChunk ? t_hi - kTChunk : 0;
    const int rows = t_hi - t_lo;
    // ---- stage [t_lo, t_hi) x [n0, n0 + kEnvTile) into LDS
    if (kVec) {
      for (int k = tid; k < rows * (kEnvTile / 4); k += kThreads) {
        const int row = k / (kEnvTile / 4), c4 = k % (kEnvTile / 4);
        const int64_t gofs = (int64_t)(t_lo + row) * N + n0 + 4 * c4;
        *(f32x4*)&s_r[row][4 * c4] = *(const f32x4*)(rew + gofs);
        *(f32x4*)&s_v[row][4 * c4] = *(const f32x4*)(val + gofs);
        *(f32x4*)&s_nv[row][4 * c4] = *(const f32x4*)(nval + gofs);
      }
      for (int k = tid; k < 2 * rows; k += kThreads) {
        const int row = k >> 1;
        const int64_t gofs = (int64_t)(t_lo + row) * N + n0;
        if (k & 1)
          *(uint4*)&s_tr[row][0] = *(const uint4*)(trunc + gofs);
        else
          *(uint4*)&s_te[row][0] = *(const uint4*)(term + gofs);
      }
    } else {
      for (int k = tid; k < rows * kEnvTile; k += kThreads) {
        const int row = k / kEnvTile, e = k % kEnvTile;
        const int n = n0 + e;
        if (n < N) {
          const int64_t gofs = (int64_t)(t_lo + row) * N + n;
          s_r[row][e] = rew[gofs];
          s_v[row][e] = val[gofs];
          s_nv[row][e] = nval[gofs];
          s_te[row][e] = term[gofs];
          s_tr[row][e] = trunc[gofs];
        }
      }
    }
    __syncthreads();
    // ---- serial backward recurrence, one lane per env
    if (tid < kEnvTile && my_n < N) {
#pragma unroll 8
      for (int row = rows - 1; row >= 0; --row) {
        const float r = s_r[row][tid];
        const float v = s_v[row][tid];
        const float te = s_te[row][tid] ? 1.0f : 0.0f;
        const float tr = s_tr[row][tid] ? 1.0f : 0.0f;
        a = gae_step(a, r, v, s_nv[row][tid], te, tr, g, c);
        s_r[row][tid] = a;      // advantage
        s_v[row][tid] = v + a;  // return (ppo.py:241)
        sum += (double)a;
        sumsq += (double)a * (double)a;
      }
    }
    __syncthreads();
    // ---- write back
    if (kVec) {
      for (int k = tid; k < rows * (kEnvTile / 4); k += kThreads) {
        const int row = k / (kEnvTile / 4), c4 = k % (kEnvTile / 4);
        const int64_t gofs = (int64_t)(t_lo + row) * N + n0 + 4 * c4;
        *(f32x4*)(adv + gofs) = *(const f32x4*)&s_r[row][4 * c4];
        *(f32x4*)(ret + gofs) = *(const f32x4*)&s_v[row][4 * c4];
      }
    } else {
      for (int k = tid; k < rows * kEnvTile; k += kThreads) {
        const int row = k / kEnvTile, e = k % kEnvTile;
        const int n = n0 + e;
        if (n < N) {
          const int64_t gofs = (int64_t)(t_lo + row) * N + n;
          adv[gofs] = s_r[row][e];
          ret[gofs] = s_v[row][e];
        }
      }
    }
    __syncthreads();
  }
  // ---- per-tile (sum, sumsq) partials, fixed reduction order (deterministic)
  if (tid < kWave) {
    for (int off = 8; off >= 1; off >>= 1) {
      sum += __shfl_down(sum, off, kEnvTile);
      sumsq += __shfl_down(sumsq, off, kEnvTile);
    }
    if (tid == 0) {
      partials[2 * blockIdx.x] = sum;
      partials[2 * blockIdx.x + 1] = sumsq;
    }
  }
}

// Sum the per-tile partials in a fixed order: dsum = {sum, sumsq}.
__global__ __launch_bounds__(256) void stats_reduce_kernel(const double* __restrict__ partials,
                                                           int n, double* __restrict__ dsum) {
  __shared__ double s0[256], s1[256];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < n; k += 256) {
    a += partials[2 * k];
    b += partials[2 * k + 1];
  }
  s0[threadIdx.x] = a;
  s1[threadIdx.x] = b;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (threadIdx.x < w) {
      s0[threadIdx.x] += s0[threadIdx.x + w];
      s1[threadIdx.x] += s1[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    dsum[0] = s0[0];
    dsum[1] = s1[0];
  }
}

// mean and unbiased std (torch.std default correction = 1), reference ppo.py:243.
__device__ __forceinline__ void mean_std_from(const double* dsum, double n, float* mean,
                                              float* std) {
  const double mu = dsum[0] / n;
  double var = (dsum[1] - dsum[0] * mu) / (n - 1.0);
  if (var < 0.0) var = 0.0;
  *mean = (float)mu;
  *std = (float)sqrt(var);
}

__global__ void stats_finalize_kernel(const double* __restrict__ dsum, double n,
                                      float* __restrict__ mean_std) {
  if (threadIdx.x == 0) mean_std_from(dsum, n, &mean_std[0], &mean_std[1]);
}

__global__ void adv_normalize_kernel(float* __restrict__ adv, const float* __restrict__ mean_std,
                                     int64_t n) {
  const float mean = mean_std[0];
  const float denom = mean_std[1] + 1e-6f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    adv[i] = (adv[i] - mean) / denom;
}

// Sample records for the minibatch gather: rec[i] = obs[0..D8) (zero padded) |
// {action bits, old log-prob, (normalised) advantage, return} | continuous actions (padded to 4).
__global__ __launch_bounds__(256) void pack_kernel(PackArgs a) {
  float mean = 0.0f, denom = 1.0f;
  if (a.advantage_norm) {
    float sd;
    mean_std_from(a.dsum, a.n_total, &mean, &sd);
    denom = sd + 1e-6f;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.B;
       i += (int64_t)gridDim.x * blockDim.x) {
    float* rec = a.rec + i * a.R;
    const float* o = a.obs + i * a.D;
    for (int k = 0; k < a.D8; k += 4) {
      f32x4 w;
      w[0] = k + 0 < a.D ? o[k + 0] : 0.0f;
      w[1] = k + 1 < a.D ? o[k + 1] : 0.0f;
      w[2] = k + 2 < a.D ? o[k + 2] : 0.0f;
      w[3] = k + 3 < a.D ? o[k + 3] : 0.0f;
      *(f32x4*)(rec + k) = w;
    }
    float adv = a.adv[i];
    if (a.advantage_norm) adv = (adv - mean) / denom;  // ppo.py:243, fp32 as the reference
    if (a.adv_out) a.adv_out[i] = adv;
    f32x4 s;
    s[0] = a.continuous ? 0.0f : __int_as_float(((const int32_t*)a.actions)[i]);
    s[1] = a.logp[i];
    s[2] = adv;
    s[3] = a.ret[i];
    *(f32x4*)(rec + a.D8) = s;
    if (a.continuous) {
      const float* act = (const float*)a.actions + i * a.A;
      for (int k = 0; k < a.A; k += 4) {
        f32x4 w;
        w[0] = k + 0 < a.A ? act[k + 0] : 0.0f;
        w[1] = k + 1 < a.A ? act[k + 1] : 0.0f;
        w[2] = k + 2 < a.A ? act[k + 2] : 0.0f;
        w[3] = k + 3 < a.A ? act[k + 3] : 0.0f;
        *(f32x4*)(rec + a.D8 + 4 + k) = w;
      }
    }
  }
}

inline int grid_for(int64_t n, int threads, int cap = 2048) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

}  // namespace

int launch_gae(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
               const float* nv, float* adv, float* ret, double* partials, int T, int N,
               float gamma, float gae_lambda, hipStream_t s, int* n_partials) {
  const int G = (N + kEnvTile - 1) / kEnvTile;
  *n_partials = G;
  if (T <= 0 || N <= 0) return DPPO_OK;
  // Python evaluates gamma * gae_lambda first, in double (ppo.py:214-216).
  const float c = (float)((double)gamma * (double)gae_lambda);
  const bool vec = (N % kEnvTile) == 0 && ((uintptr_t)r % 16 == 0) && ((uintptr_t)v % 16 == 0) &&
                   ((uintptr_t)nv % 16 == 0) && ((uintptr_t)adv % 16 == 0) &&
                   ((uintptr_t)ret % 16 == 0) && ((uintptr_t)te % 16 == 0) &&
                   ((uintptr_t)tr % 16 == 0);
  if (vec)
    hipLaunchKernelGGL(gae_kernel<true>, dim3(G), dim3(kThreads), 0, s, r, te, tr, v, nv, adv, ret,
                       partials, T, N, gamma, c);
  else
    hipLaunchKernelGGL(gae_kernel<false>, dim3(G), dim3(kThreads), 0, s, r, te, tr, v, nv, adv,
                       ret, partials, T, N, gamma, c);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_stats_reduce(const double* partials, int n_partials, double* dsum, hipStream_t s) {
  hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(256), 0, s, partials, n_partials, dsum);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_stats_finalize(const double* dsum, double n_total, float* mean_std, hipStream_t s) {
  hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(64), 0, s, dsum, n_total, mean_std);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_adv_normalize(float* adv, const float* mean_std, int64_t n, hipStream_t s) {
  if (n <= 0) return DPPO_OK;
  hipLaunchKernelGGL(adv_normalize_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, adv,
                     mean_std, n);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.B <= 0) return DPPO_OK;
  hipLaunchKernelGGL(pack_kernel, dim3(grid_for(a.B, 256)), dim3(256), 0, s, a);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
