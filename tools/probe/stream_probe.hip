// Timing probe (not part of libdppo): the pure data movement of the GAE at its layout, no scan.
// adv = r + v, ret = nv + te + tr per element (22 B/elem), 16-B vector accesses, grid-stride.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-B store written through to memory (sc1: the line leaves the XCD's L2 while the kernel runs
// instead of as a dirty line at the kernel boundary; MI355X_MICROARCH.md publish-large)
__device__ __forceinline__ void store_wt(f32x4* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <bool WT>
__global__ __launch_bounds__(256) void stream_kernel(const float* __restrict__ r,
                                                     const uint8_t* __restrict__ te,
                                                     const uint8_t* __restrict__ tr,
                                                     const float* __restrict__ v,
                                                     const float* __restrict__ nv,
                                                     float* __restrict__ adv,
                                                     float* __restrict__ ret, int64_t n4) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 a = ((const f32x4*)r)[i];
    const f32x4 b = ((const f32x4*)v)[i];
    const f32x4 c = ((const f32x4*)nv)[i];
    const uint32_t t = ((const uint32_t*)te)[i];
    const uint32_t u = ((const uint32_t*)tr)[i];
    f32x4 o = c;
    o[0] += (float)((t ^ u) & 0xff);
    if (WT) {
      store_wt((f32x4*)adv + i, a + b);
      store_wt((f32x4*)ret + i, o);
    } else {
      ((f32x4*)adv)[i] = a + b;
      ((f32x4*)ret)[i] = o;
    }
  }
}

extern "C" int probe_stream(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
                            const float* nv, float* adv, float* ret, int64_t n, int grid,
                            void* stream, int write_through) {
  if (write_through)
    hipLaunchKernelGGL(stream_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, r, te,
                       tr, v, nv, adv, ret, n / 4);
  else
    hipLaunchKernelGGL(stream_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, r, te,
                       tr, v, nv, adv, ret, n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
