// Timing probe (not part of libdppo): issue rate of v_mfma_f32_16x16x4_f32 chains on gfx950.
// Each wave runs `iters` rounds of NACC independent accumulator chains (operands in registers);
// s_memtime brackets the loop.  Launch with 4 * waves_per_simd waves per workgroup, one workgroup
// per CU, to see how two waves on a SIMD share the matrix pipe.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(512) void mfma_chain(float* out, long long* cyc, int iters,
                                                  int active_waves) {
  const int wave = threadIdx.x >> 6;
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, (float)threadIdx.x};
  float a = 1.0f + threadIdx.x * 1e-3f, b = 0.5f;
  long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < active_waves) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < NACC; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    cyc[blockIdx.x * 8 + wave] = t1 - t0;
    if (blockIdx.x == 0) {  // absolute stamps of block 0 (overlap of its waves)
      cyc[gridDim.x * 8 + 2 * wave] = t0;
      cyc[gridDim.x * 8 + 2 * wave + 1] = t1;
    }
  }
}

extern "C" int probe_mfma(int nacc, float* out, long long* cyc, int iters, int waves,
                          int active_waves, int blocks, void* stream) {
  dim3 g(blocks), b(waves * 64);
  hipStream_t s = (hipStream_t)stream;
  switch (nacc) {
    case 1: hipLaunchKernelGGL(mfma_chain<1>, g, b, 0, s, out, cyc, iters, active_waves); break;
    case 2: hipLaunchKernelGGL(mfma_chain<2>, g, b, 0, s, out, cyc, iters, active_waves); break;
    case 4: hipLaunchKernelGGL(mfma_chain<4>, g, b, 0, s, out, cyc, iters, active_waves); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Does VALU work co-issue with fp32 MFMAs on one SIMD?  Each active wave runs 4 MFMA accumulator
// chains and NV independent v_fma_f32 chains per MFMA (mode 0); mode 1 splits the two across the
// two waves of each SIMD (waves 0-3: MFMAs only, waves 4-7: the same VALU work only).
template <int NV>
__global__ __launch_bounds__(512) void mfma_valu(float* out, long long* cyc, int iters, int mode) {
  const int wave = threadIdx.x >> 6;
  f32x4 acc[4];
  float x[8];
  for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, (float)threadIdx.x};
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3f + i;
  float a = 1.0f + threadIdx.x * 1e-3f, b = 0.5f, c = 0.999f, d = 1e-3f;
  const int w = __builtin_amdgcn_readfirstlane(wave);
  const int role = mode == 0 ? 0 : (w < 4 ? 1 : 2);  // 0: both, 1: MFMA only, 2: VALU only
  long long t0 = __builtin_amdgcn_s_memtime();
  if (role == 0) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
          for (int v = 0; v < NV; ++v) x[v] = __builtin_fmaf(x[v], c, d);
        }
    }
  } else if (role == 1) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int v = 0; v < NV; ++v) x[v] = __builtin_fmaf(x[v], c, d);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += x[i];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

extern "C" int probe_mfma_valu(int nv, int mode, float* out, long long* cyc, int iters, int blocks,
                               void* stream) {
  dim3 g(blocks), b(mode == 0 ? 256 : 512);
  hipStream_t s = (hipStream_t)stream;
  switch (nv) {
    case 0: hipLaunchKernelGGL(mfma_valu<0>, g, b, 0, s, out, cyc, iters, mode); break;
    case 1: hipLaunchKernelGGL(mfma_valu<1>, g, b, 0, s, out, cyc, iters, mode); break;
    case 2: hipLaunchKernelGGL(mfma_valu<2>, g, b, 0, s, out, cyc, iters, mode); break;
    case 4: hipLaunchKernelGGL(mfma_valu<4>, g, b, 0, s, out, cyc, iters, mode); break;
    case 6: hipLaunchKernelGGL(mfma_valu<6>, g, b, 0, s, out, cyc, iters, mode); break;
    case 8: hipLaunchKernelGGL(mfma_valu<8>, g, b, 0, s, out, cyc, iters, mode); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Round 4: the issue cost of one VALU instruction beside the MFMA chains, by instruction kind
// (KIND 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_exp_f32, 3 v_add_f32, 4 v_pk_add_f32, 5 v_pk_mul_f32,
// 6 v_rcp_f32); MODE 0: NV per MFMA on the MFMA wave, MODE 2: the VALU stream alone (no MFMA).
typedef float f32x2p __attribute__((ext_vector_type(2)));
template <int KIND>
__device__ __forceinline__ void valu_op(f32x2p& x, f32x2p c, f32x2p d) {
  if (KIND == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[0]) : "v"(c[0]), "v"(d[0]));
  if (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(d));
  if (KIND == 2) asm volatile("v_exp_f32 %0, %0" : "+v"(x[0]));
  if (KIND == 3) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[0]) : "v"(d[0]));
  if (KIND == 4) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(d));
  if (KIND == 5) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(c));
  if (KIND == 6) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[0]));
}

template <int KIND, int NV, int MODE>
__global__ __launch_bounds__(256) void mfma_kind(float* out, long long* cyc, int iters) {
  const int wave = threadIdx.x >> 6;
  f32x4 acc[4];
  f32x2p x[8];
  for (int i = 0; i < 4; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, (float)threadIdx.x};
  for (int i = 0; i < 8; ++i) x[i] = (f32x2p){threadIdx.x * 1e-3f + i, 0.5f + i};
  const float a = 1.0f + threadIdx.x * 1e-3f, b = 0.5f;
  const f32x2p c = {0.999f, 0.998f}, d = {1e-3f, 2e-3f};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (MODE == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
        // round-robin over 8 independent chains: throughput, not one chain's latency
#pragma unroll
        for (int v = 0; v < NV; ++v) valu_op<KIND>(x[((4 * j + i) * NV + v) & 7], c, d);
      }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += x[i][0] + x[i][1];
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

#define KCASE(K, N)                                                                   \
  case K * 16 + N:                                                                    \
    if (mode == 0) hipLaunchKernelGGL((mfma_kind<K, N, 0>), g, b, 0, s, out, cyc, iters); \
    else hipLaunchKernelGGL((mfma_kind<K, N, 2>), g, b, 0, s, out, cyc, iters);          \
    break;
#define KROW(K) KCASE(K, 1) KCASE(K, 2) KCASE(K, 4) KCASE(K, 8)
extern "C" int probe_mfma_kind(int kind, int nv, int mode, float* out, long long* cyc, int iters,
                               int blocks, void* stream) {
  dim3 g(blocks), b(256);
  hipStream_t s = (hipStream_t)stream;
  switch (kind * 16 + nv) {
    KROW(0) KROW(1) KROW(2) KROW(3) KROW(4) KROW(5) KROW(6)
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
