// Timing probe (not part of libdppo): variants of the GAE launch's pure data movement (22 B per
// element at [T][N]: read r, v, nv (16 B per lane) and the two flag bytes, write adv and ret), to
// find what bounds one 23 MB launch at N = 8192.  MODE bits:
//   1  non-temporal loads and stores (__builtin_nontemporal_load / _store: the nt cache policy)
//   2  two elements per thread (i and i + n4 / 2: more bytes in flight per wave, half the waves)
//   4  XCD-contiguous blocks: block b works on slice (b % 8) * (grid / 8) + b / 8, so that the
//      blocks one XCD runs (round-robin dispatch) touch one contiguous eighth of every buffer
#include <hip/hip_runtime.h>
#include <cstdint>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if (MODE & 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int MODE, typename T>
__device__ __forceinline__ void st(T* p, T v) {
  if (MODE & 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int MODE>
__global__ __launch_bounds__(256) void stream2_kernel(const float* __restrict__ r,
                                                      const uint8_t* __restrict__ te,
                                                      const uint8_t* __restrict__ tr,
                                                      const float* __restrict__ v,
                                                      const float* __restrict__ nv,
                                                      float* __restrict__ adv,
                                                      float* __restrict__ ret, int64_t n4) {
  const int64_t g = gridDim.x;
  int64_t b = blockIdx.x;
  if (MODE & 4) b = (b % 8) * (g / 8) + b / 8;
  constexpr int E = (MODE & 2) ? 2 : 1;
  const int64_t per = n4 / E;
  for (int64_t i = b * 256 + threadIdx.x; i < per; i += g * 256) {
    f32x4 a[E], bb[E], c[E];
    uint32_t t[E], u[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t k = i + e * per;
      a[e] = ld<MODE>((const f32x4*)r + k);
      bb[e] = ld<MODE>((const f32x4*)v + k);
      c[e] = ld<MODE>((const f32x4*)nv + k);
      t[e] = ld<MODE>((const uint32_t*)te + k);
      u[e] = ld<MODE>((const uint32_t*)tr + k);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t k = i + e * per;
      f32x4 o = c[e];
      o[0] += (float)((t[e] ^ u[e]) & 0xff);
      st<MODE>((f32x4*)adv + k, a[e] + bb[e]);
      st<MODE>((f32x4*)ret + k, o);
    }
  }
}

extern "C" int probe_stream2(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
                             const float* nv, float* adv, float* ret, int64_t n, int grid,
                             void* stream, int mode) {
  const hipStream_t s = (hipStream_t)stream;
  const int64_t n4 = n / 4;
#define CASE(M)                                                                                \
  case M:                                                                                      \
    hipLaunchKernelGGL(stream2_kernel<M>, dim3(grid), dim3(256), 0, s, r, te, tr, v, nv, adv, \
                       ret, n4);                                                               \
    break;
  switch (mode) {
    CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7)
    default: return -1;
  }
#undef CASE
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
