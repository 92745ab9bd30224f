// Fisher-Yates resolution on the device: minibatch permutations from their swap targets.
//
// np.random.permutation(n) (reference diamond/ppo.py:254; numpy legacy RandomState) is the
// sequential shuffle   a = arange(n); for i = n-1 .. 1: swap(a[i], a[j_i])   with j_i <= i drawn
// from MT19937 by rejection (perm.cpp draws the j_i on the host, bit-exactly).  The swaps are a
// dependent chain on the host (~1.4 ms per 4 x 524288 on a 5 GHz core); here they are resolved
// in parallel with the closed form of the shuffle:
//
//   position i is final after step i, and before step i position p < i holds the value last
//   written into it, i.e. by the latest step i'' > i with j_i'' = p (or p itself if none).
//   With  succ(i) = min{ i'' > i : j_i'' = j_i }   and   M(q) = min{ i'' > q : j_i'' = q }:
//     W(q)   = value at position q just before step q = root(q)  (follow M until it is absent)
//     out[i] = succ(i) exists ? W(succ(i)) : j_i          (i >= 1)
//     out[0] = W(0)
//
// Three grid-stride passes over count*n elements (HBM/L2-latency bound, no MFMA):
//   build : per-target linked lists   head[c][p] <- i   (atomicExch; list order irrelevant)
//   links : M(x) from bucket x, succ(x) from bucket j_x   (bucket sizes ~ ln(n/p), tiny)
//   solve : out = W(succ) / j / W(0)   (chains strictly increase, length ~ ln n)
// Every value is a min over a set, so the result is deterministic despite the atomics.
#include "common.h"

namespace dppo {
namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void fy_build_kernel(const int32_t* __restrict__ tgt,
                                                         int32_t* __restrict__ head,
                                                         int32_t* __restrict__ nxt, int64_t n,
                                                         int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int32_t i = (int32_t)(g - c * n);
    const int32_t p = tgt[g];
    int32_t prev = -1;
    // i = 0 takes no step; a target outside [0, i] (never produced by the host draw) is ignored
    // rather than allowed to index out of range
    if (i > 0 && (uint32_t)p <= (uint32_t)i) prev = atomicExch(&head[c * n + p], i);
    nxt[g] = prev;
  }
}

__device__ __forceinline__ int32_t min_above(const int32_t* __restrict__ head,
                                             const int32_t* __restrict__ nxt, int64_t base,
                                             int32_t bucket, int32_t x) {
  int32_t best = 0x7FFFFFFF;
  for (int32_t it = head[base + bucket]; it >= 0; it = nxt[base + it])
    best = (it > x && it < best) ? it : best;
  return best == 0x7FFFFFFF ? -1 : best;
}

__global__ __launch_bounds__(kBlock) void fy_links_kernel(const int32_t* __restrict__ tgt,
                                                         const int32_t* __restrict__ head,
                                                         const int32_t* __restrict__ nxt,
                                                         int32_t* __restrict__ mq,
                                                         int32_t* __restrict__ succ, int64_t n,
                                                         int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int64_t base = c * n;
    const int32_t x = (int32_t)(g - base);
    mq[g] = min_above(head, nxt, base, x, x);
    int32_t s = -1;
    const int32_t p = tgt[g];
    if (x > 0 && (uint32_t)p <= (uint32_t)x) s = min_above(head, nxt, base, p, x);
    succ[g] = s;
  }
}

__device__ __forceinline__ int32_t root(const int32_t* __restrict__ mq, int64_t base, int32_t q) {
  for (int32_t m = mq[base + q]; m >= 0; m = mq[base + q]) q = m;
  return q;
}

// out aliases succ (each thread reads its own succ before overwriting it)
__global__ __launch_bounds__(kBlock) void fy_solve_kernel(const int32_t* __restrict__ tgt,
                                                         const int32_t* __restrict__ mq,
                                                         int32_t* out, int64_t n, int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int64_t base = c * n;
    const int32_t x = (int32_t)(g - base);
    int32_t v;
    if (x == 0) {
      v = root(mq, base, 0);
    } else {
      const int32_t s = out[g];
      v = s >= 0 ? root(mq, base, s) : tgt[g];
    }
    out[g] = v;
  }
}

int fy_grid(int64_t total) {
  int64_t b = (total + kBlock - 1) / kBlock;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

int launch_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                        int32_t* scratch, hipStream_t s) {
  const int64_t total = n * (int64_t)count;
  if (total == 0) return DPPO_OK;
  int32_t* head = scratch;
  int32_t* nxt = scratch + total;
  int32_t* mq = scratch + 2 * total;
  DPPO_HIP_CHECK(hipMemsetAsync(head, 0xFF, (size_t)total * sizeof(int32_t), s));
  const int G = fy_grid(total);
  DPPO_LAUNCH(fy_build_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, n, total);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(fy_links_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, mq, perms, n, total);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(fy_solve_kernel, dim3(G), dim3(kBlock), 0, s, targets, mq, perms, n, total);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
