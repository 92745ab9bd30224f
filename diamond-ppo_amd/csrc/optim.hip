// Gradient slab reduction, clip_grad_norm_ and Adam on gfx950.
//
// Replaces, per minibatch, loss.backward()'s parameter-gradient accumulation (ppo.py:283),
// nn.utils.clip_grad_norm_(params, 0.5) (ppo.py:284; torch nn/utils/clip_grad.py:96,106,165,169)
// and optimizer.step() (ppo.py:285; torch optim/adam.py _single_tensor_adam, the CPU path the
// reference runs: step += 1; exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
// denom = sqrt(exp_avg_sq)/sqrt(bc2) + eps; p.addcdiv_(exp_avg, denom, -lr/bc1)).
//
// Both kernels are latency-bound, not bandwidth-bound (the slabs are G x P floats, ~13 MB at
// G = 256; P ~ 13-14 K), so every thread keeps many independent loads in flight:
//  * slab_reduce: one workgroup per 64 parameters; each of its 16 waves sums every 16th slab
//    for the 64 parameters (lane = parameter, 256 contiguous bytes per wave load, all 16 of a
//    wave's loads in flight at once at G = 256: one memory round trip instead of the four a
//    4-wave block needs), the 16 partials are combined through LDS in a fixed order
//    (bit-reproducible), and each block also emits its partial sum of squares.
//  * clip_adam: the global norm comes from those per-block partials (fixed order) or, after an
//    RCCL all-reduce changed the gradient, from the gradient itself with 8 loads in flight.
#include "common.h"

namespace dppo {
namespace {

constexpr int kRedParams = 64;  // parameters per slab_reduce workgroup

#ifdef DPPO_RA_TRACE
// per block of reduce_adam_kernel: s_memrealtime at entry, slabs summed, published, released, end
__device__ long long g_ra_edges[512][5];
#define RA_EDGE(i) \
  if (threadIdx.x == 0 && blockIdx.x < 512) \
    g_ra_edges[blockIdx.x][i] = (long long)__builtin_amdgcn_s_memrealtime()
#else
#define RA_EDGE(i)
#endif
#ifndef DPPO_RA_WAVES
#define DPPO_RA_WAVES 16
#endif
constexpr int kRedWaves = DPPO_RA_WAVES;  // (A/B: DPPO_RA_WAVES=8, twice the loads per wave)
constexpr int kSlabBatch = 256 / kRedWaves;  // one batch of loads in flight per lane: G = 256
constexpr int kRedThreads = kRedWaves * 64;

// Sum of slabs[g][p] over g for this block's 64 parameters (lane = parameter): wave w takes slabs
// w, w + kRedWaves, ... in order, all kSlabBatch loads in flight; the wave partials are combined by wave 0 in
// wave order.  Returns the total in wave 0 (other waves: 0).
__device__ __forceinline__ float slab_sum(const float* __restrict__ slabs, int G, int64_t stride,
                                          int64_t p, int64_t n, float (*part)[kRedParams]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float s = 0.0f;
  if (p < n) {
    const float* src = slabs + p;
    int g = wave;
    for (; g + (kSlabBatch - 1) * kRedWaves < G; g += kSlabBatch * kRedWaves) {
      float x[kSlabBatch];
#pragma unroll
      for (int k = 0; k < kSlabBatch; ++k) {
        // Non-temporal slab reads (each slab float is read once).  They cost this kernel
        // ~0.1-0.25 us, and the next minibatch kernel launch gains: C2 53.3 -> 51.4-51.5 us (0.593
        // -> 0.614 of peak), C4 59.7-59.9 -> 58.8-58.9 us, C3 / C5 unchanged (tools/gpu/
        // r05_ra_nt2.sh, 2 A/B pairs) -- the slab lines no longer displace what that launch
        // re-reads from L2.  -DDPPO_RA_PLAIN restores plain reads (A/B).
#ifdef DPPO_RA_PLAIN
        x[k] = src[(int64_t)(g + kRedWaves * k) * stride];
#else
        x[k] = __builtin_nontemporal_load(src + (int64_t)(g + kRedWaves * k) * stride);
#endif
      }
#pragma unroll
      for (int k = 0; k < kSlabBatch; ++k) s += x[k];
    }
    for (; g < G; g += kRedWaves) s += src[(int64_t)g * stride];
  }
  part[wave][lane] = s;
  __syncthreads();
  float t = 0.0f;
  if (wave == 0) {
#pragma unroll
    for (int w = 0; w < kRedWaves; ++w) t += part[w][lane];
  }
  return t;
}

__global__ __launch_bounds__(kRedThreads) void slab_reduce_kernel(
    const float* __restrict__ slabs, int G, int64_t stride, int64_t p_total,
    float* __restrict__ grad, double* __restrict__ sq_part, int64_t ls_off, int ls_n,
    float ent_coef, int add_entropy_const) {
  __shared__ float part[kRedWaves][kRedParams];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * kRedParams + lane;
  const int64_t n = p_total + 8;
  float t = slab_sum(slabs, G, stride, p, n, part);
  if (wave == 0) {
    // d(-beta * mean H)/d log_std = -beta per action dim (continuous_ppo.py:286-291): a
    // constant the per-sample kernel does not see; added once (rank 0 under data parallelism).
    if (add_entropy_const && p >= ls_off && p < ls_off + ls_n) t -= ent_coef;
    if (p < n) grad[p] = t;
    double q = (p < p_total) ? (double)t * (double)t : 0.0;
    for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
    if (lane == 0) sq_part[blockIdx.x] = q;
  }
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

// One Adam element in torch _single_tensor_adam's op order (no FMA contraction).
__device__ __forceinline__ void adam_elem(float* __restrict__ params, const float* __restrict__ grad,
                                          float* __restrict__ m, float* __restrict__ v,
                                          int64_t k, float coef, float w1, float w2, float beta2,
                                          float bc2_sqrt, float eps, float neg_step_size) {
#pragma clang fp contract(off)
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

// grad: [n] flat gradient followed by 8 loss slots {sum l_pi, sum l_v, sum H, ...}.
// sq_part/n_sq: per-block partial sums of squares of grad (null => recompute from grad).
__global__ __launch_bounds__(256) void clip_adam_kernel(
    float* __restrict__ params, float* __restrict__ grad, float* __restrict__ m,
    float* __restrict__ v, int64_t n, const double* __restrict__ sq_part, int n_sq,
    float max_norm, float neg_step_size, float bc2_sqrt, float beta1, float beta2, float eps,
    float* __restrict__ out_norm, float* __restrict__ trace, float inv_m, float vf, float ent) {
#pragma clang fp contract(off)
  __shared__ double sh[4];
  double sq = 0.0;
  if (sq_part) {
    for (int k = threadIdx.x; k < n_sq; k += blockDim.x) sq += sq_part[k];
  } else {
    int64_t k = threadIdx.x;
    for (; k + 7 * 256 < n; k += 8 * 256) {
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = grad[k + j * 256];
#pragma unroll
      for (int j = 0; j < 8; ++j) sq += (double)g[j] * (double)g[j];
    }
    for (; k < n; k += 256) sq += (double)grad[k] * (double)grad[k];
  }
  const double tot = block_sum(sq, sh);
  float norm;
  const float coef = clip_coef(tot, max_norm, &norm);
  const float w1 = 1.0f - beta1;
  const float w2 = 1.0f - beta2;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    adam_elem(params, grad, m, v, k, coef, w1, w2, beta2, bc2_sqrt, eps, neg_step_size);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (out_norm) *out_norm = norm;
    if (trace) write_trace(trace, grad[n], grad[n + 1], grad[n + 2], norm, inv_m, vf, ent);
  }
}

// Slab reduction + clip_grad_norm_ + Adam in ONE launch (single device).  Every block reduces its
// 64 parameters as slab_reduce_kernel does, then wave 0 publishes the block's sum of squares as
// one tagged 64-bit word {launch epoch, float partial} (the block covering the loss slots also
// publishes those three sums the same way) and polls every block's word until all carry this
// launch's epoch: the data is its own arrival flag, so the wait costs no counter atomics, no
// release word and no second round trip to fetch the partials (tools/ra_trace.py: the counter
// fan-in took ~1.7 us from publish to release, the reads after it ~0.5 us more).  Every block then
// sums the same partials in the same order (bit-reproducible global norm) and applies Adam to its
// own 64 parameters, whose gradients it still holds in registers and whose moments it prefetched
// before the wait; the other 15 waves leave once the slabs are summed.  Words are read and written
// with agent-scope atomics (sc1: no stale L2 line, no acquire fence).  Tags are monotonic per
// handle (launch `epoch` >= 1, words zeroed at handle creation), so nothing is reset.
// Co-residency of the ~210 blocks of 1024 threads is checked once per handle
// (reduce_adam_capacity; a device that cannot hold them all takes the three-kernel path instead),
// and the wait is bounded: a block whose wait times out leaves its parameters untouched and raises
// the handle's sticky error word, which the next C-ABI call reports -- never a silently stale norm.
constexpr int kTagWordsPerLane = 16;  // tagged words a polling lane holds: blocks + 3 <= 1024

__device__ __forceinline__ unsigned long long tag_word(unsigned epoch, float x) {
  return ((unsigned long long)epoch << 32) | __float_as_uint(x);
}

__global__ __launch_bounds__(kRedThreads) void reduce_adam_kernel(
    const float* __restrict__ slabs, int G, int64_t stride, int64_t p_total, float* grad,
    unsigned long long* tags, int64_t ls_off, int ls_n, float ent_coef, int add_entropy_const,
    unsigned epoch, float* __restrict__ params, float* __restrict__ m,
    float* __restrict__ v, float max_norm, float neg_step_size, float bc2_sqrt, float beta1,
    float beta2, float eps, float* __restrict__ trace, float inv_m, float vf, float ent,
    unsigned* err, unsigned long long timeout_ticks, PeerArgs pl) {
#pragma clang fp contract(off)
  __shared__ float part[kRedWaves][kRedParams];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * kRedParams + lane;
  const int64_t n = p_total + 8;
  const int nb = (int)gridDim.x, nw = nb + 3;  // words: one per block, then the 3 loss sums
  // this block's Adam operands, loaded while the slabs stream in
  float mk = 0.f, vk = 0.f, pk = 0.f;
  RA_EDGE(0);
  if (wave == 0 && p < p_total) {
    mk = m[p];
    vk = v[p];
    pk = params[p];
  }
  float t = slab_sum(slabs, G, stride, p, n, part);
  RA_EDGE(1);
  if (wave != 0) return;
  if (add_entropy_const && p >= ls_off && p < ls_off + ls_n) t -= ent_coef;
  if (pl.world > 0) {
    // data parallel over a peer exchange: publish this block's 64 sums as tagged words {seq,
    // value} in this rank's buffer (the data is its own arrival flag: one system-scope store, no
    // drain, no flag round trip), poll word p of every rank until it carries this exchange's
    // tag, and sum in rank order (the same bits on every rank) -- the cross-rank step of the
    // minibatch, inside this launch
    if (p < n) peer_put(peer_tagged(pl, pl.rank) + p, tag_word(pl.seq, t));
    float x[kMaxPeers];
    unsigned pend = 0;
#pragma unroll
    for (int r = 0; r < kMaxPeers; ++r) {
      x[r] = 0.f;
      if (r < pl.world && p < n) pend |= 1u << r;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long seen = 0;  // the last word read of the lowest rank still pending
    for (unsigned k = 0;; ++k) {
      if (pl.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#pragma unroll
      for (int r = kMaxPeers - 1; r >= 0; --r) {
        if (pend & (1u << r)) {
          const unsigned long long w = peer_get(peer_tagged(pl, r) + p);
          if ((unsigned)(w >> 32) == pl.seq) {
            x[r] = __uint_as_float((unsigned)w);
            pend &= ~(1u << r);
          } else {
            seen = w;
          }
        }
      }
      if (__ballot(pend != 0) == 0) break;
      __builtin_amdgcn_s_sleep(1);
      if ((k & 255u) == 255u) {
        const bool late = __builtin_amdgcn_s_memrealtime() - t0 > pl.timeout_ticks;
        if (late || err_set(err)) {
          if (late) {  // the first lane still waiting names the rank and the word
            const unsigned long long b = __ballot(pend != 0);
            const int l = __ffsll((long long)b) - 1;
            const unsigned pr = (unsigned)__shfl((int)pend, l);
            const unsigned r = (unsigned)(__ffs((int)pr) - 1);
            if (lane == l) raise_err_seen(err, err_word(kErrPeerTimeout, r, (unsigned)p), seen);
          }
          return;  // parameters untouched; the handle reports the error
        }
      }
    }
    t = x[0];
#pragma unroll
    for (int r = 1; r < kMaxPeers; ++r)
      if (r < pl.world) t += x[r];
  }
  if (p < n) grad[p] = t;
  // (wave sums by DPP row moves + 4 lane reads: the 6-step __shfl_xor butterfly on doubles was
  // 12 LDS-crossbar round trips, ~0.3 us of the launch, here and in the norm below)
  const double q = wave_sum_f64((p < p_total) ? (double)t * (double)t : 0.0);
  if (lane == 0)
    __hip_atomic_store(tags + blockIdx.x, tag_word(epoch, (float)q), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (p >= p_total && p < p_total + 3)
    __hip_atomic_store(tags + nb + (p - p_total), tag_word(epoch, t), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  RA_EDGE(2);
  // poll: each lane keeps its words' loads in flight together; the loop exit is wave-uniform
  unsigned long long w[kTagWordsPerLane];
  unsigned pending = 0;
#pragma unroll
  for (int j = 0; j < kTagWordsPerLane; ++j) {
    w[j] = 0;
    if (j * 64 + lane < nw) pending |= 1u << j;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned k = 0;; ++k) {
#pragma unroll
    for (int j = 0; j < kTagWordsPerLane; ++j)
      if (pending & (1u << j))
        w[j] = __hip_atomic_load(tags + j * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < kTagWordsPerLane; ++j)
      if ((unsigned)(w[j] >> 32) == epoch) pending &= ~(1u << j);
    if (__ballot(pending != 0) == 0) break;
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255u) == 255u) {
      // with a peer exchange in front, this wait's bound starts after the peer wait's has run
      // out: a block stuck on a peer word then reports as a peer timeout (code 2 + rank + word)
      // instead of its siblings reporting the tag wait it caused (round-5 diagnosis)
      const bool late = __builtin_amdgcn_s_memrealtime() - t0 >
                        timeout_ticks + (pl.world > 0 ? pl.timeout_ticks : 0ull);
      if (late || err_set(err)) {
        if (late) {  // the first word still missing: the block index (or nb + loss slot)
          unsigned first = 0xffffu;
#pragma unroll
          for (int j = kTagWordsPerLane - 1; j >= 0; --j)
            if (pending & (1u << j)) first = (unsigned)(j * 64 + lane);
          const unsigned long long b = __ballot(pending != 0);
          unsigned lo = 0xffffu;
          for (unsigned long long bb = b; bb; bb &= bb - 1) {
            const int l = __ffsll((long long)bb) - 1;
            const unsigned f = (unsigned)__shfl((int)first, l);
            lo = f < lo ? f : lo;
          }
          if (lane == 0) raise_err(err, err_word(kErrTagTimeout, blockIdx.x & 0xffu, lo));
        }
        return;  // parameters untouched; the next C-ABI call reports the error
      }
    }
  }
  RA_EDGE(3);
  // global norm: every block sums the same per-block squares in the same order
  double sq = 0.0;
#pragma unroll
  for (int j = 0; j < kTagWordsPerLane; ++j)
    if (j * 64 + lane < nb) sq += (double)__uint_as_float((unsigned)w[j]);
  sq = wave_sum_f64(sq);
  float norm;
  const float coef = clip_coef(sq, max_norm, &norm);
  if (p < p_total) {
    adam_regs(pk, t, mk, vk, coef, 1.0f - beta1, 1.0f - beta2, beta2, bc2_sqrt, eps,
              neg_step_size);
    params[p] = pk;
    m[p] = mk;
    v[p] = vk;
  }
#ifdef DPPO_RA_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RA_EDGE(4);
#endif
  if (blockIdx.x == 0 && trace) {
    // the loss sums: words nb .. nb + 2 (lane (nb + i) % 64, slot (nb + i) / 64)
    float s[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int wi = nb + i, ji = wi >> 6;
      float x = 0.f;
#pragma unroll
      for (int j = 0; j < kTagWordsPerLane; ++j)
        if (j == ji) x = __uint_as_float((unsigned)w[j]);
      s[i] = __shfl(x, wi & 63);
    }
    if (lane == 0) write_trace(trace, s[0], s[1], s[2], norm, inv_m, vf, ent);
  }
}

// dppo_fanin_selftest: `gridDim.x` workgroups meet in one grid_fanin; the dynamic LDS they hold
// only limits how many fit on a CU, so a test can launch a grid that cannot be co-resident.
__global__ __launch_bounds__(1024) void fanin_probe_kernel(unsigned* ctr, unsigned* err,
                                                           unsigned long long timeout_ticks) {
  extern __shared__ float hold[];
  if (threadIdx.x == 0) {
    hold[0] = 0.0f;
    (void)grid_fanin(ctr, 1u, timeout_ticks, err);
  }
  __syncthreads();
}

template <typename F>
__global__ __launch_bounds__(256) void rank_sum_kernel(RankPtrs src, int n, F* __restrict__ out,
                                                       int64_t count) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    F acc = ((const F*)src.p[0])[i];
    for (int r = 1; r < n; ++r) acc += ((const F*)src.p[r])[i];
    out[i] = acc;
  }
}

}  // namespace

#ifdef DPPO_RA_TRACE
extern "C" __attribute__((visibility("default"))) int dppo_debug_ra_edges(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ra_edges), sizeof(g_ra_edges)) == hipSuccess ? 0 : -1;
}
#endif

int launch_rank_sum(const RankPtrs& src, int n, void* out, int64_t count, bool f64,
                    hipStream_t s) {
  int64_t g = (count + 255) / 256;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  if (f64)
    DPPO_LAUNCH(rank_sum_kernel<double>, dim3((unsigned)g), dim3(256), 0, s, src, n,
                (double*)out, count);
  else
    DPPO_LAUNCH(rank_sum_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, src, n,
                (float*)out, count);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int slab_reduce_blocks(int64_t p_total) { return (int)((p_total + 8 + kRedParams - 1) / kRedParams); }

int launch_slab_reduce(const float* slabs, int G, int64_t slab_stride, int64_t p_total,
                       float* grad, double* sq_part, int64_t ls_off, int ls_n, float ent_coef,
                       int add_entropy_const, hipStream_t s) {
  DPPO_LAUNCH(slab_reduce_kernel, dim3(slab_reduce_blocks(p_total)), dim3(kRedThreads), 0, s,
                     slabs, G, slab_stride, p_total, grad, sq_part, ls_off, ls_n, ent_coef,
                     add_entropy_const);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_clip_adam_traced(float* params, float* grad, float* m, float* v, int64_t n,
                            const double* sq_part, int n_sq, float max_norm, float neg_step_size,
                            float bc2_sqrt, float beta1, float beta2, float eps, float* out_norm,
                            float* trace, float inv_m, float vf, float ent, hipStream_t s) {
  int64_t g = (n + 255) / 256;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  DPPO_LAUNCH(clip_adam_kernel, dim3((unsigned)g), dim3(256), 0, s, params, grad, m, v, n,
                     sq_part, n_sq, max_norm, neg_step_size, bc2_sqrt, beta1, beta2, eps,
                     out_norm, trace, inv_m, vf, ent);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_reduce_adam(const float* slabs, int G, int64_t slab_stride, int64_t p_total, float* grad,
                       unsigned long long* tags, int64_t ls_off, int ls_n, float ent_coef,
                       int add_entropy_const, unsigned epoch, float* params,
                       float* m, float* v, float max_norm, float neg_step_size, float bc2_sqrt,
                       float beta1, float beta2, float eps, float* trace, float inv_m, float vf,
                       float ent, unsigned* err, unsigned long long timeout_ticks, hipStream_t s,
                       const PeerArgs* peer) {
  PeerArgs pl{};
  if (peer) {
    pl = *peer;
    if ((p_total + 8) * 8 > pl.data_bytes) {
      set_error("peer exchange: %lld gradient values exceed the exchange buffer",
                (long long)(p_total + 8));
      return DPPO_EUNSUPPORTED;
    }
  }
  DPPO_LAUNCH(reduce_adam_kernel, dim3(reduce_adam_blocks(p_total)), dim3(kRedThreads), 0, s, slabs, G,
              slab_stride, p_total, grad, tags, ls_off, ls_n, ent_coef, add_entropy_const,
              epoch, params, m, v, max_norm, neg_step_size, bc2_sqrt, beta1, beta2, eps,
              trace, inv_m, vf, ent, err, timeout_ticks, pl);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int reduce_adam_blocks(int64_t p_total) { return slab_reduce_blocks(p_total); }

int reduce_adam_tag_words(int64_t p_total) { return reduce_adam_blocks(p_total) + 3; }

int reduce_adam_capacity(int device, int64_t p_total) {
  if (reduce_adam_tag_words(p_total) > 64 * kTagWordsPerLane) return 0;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)reduce_adam_kernel,
                                                   kRedThreads, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return per_cu * cus;
}

int launch_fanin_probe(int blocks, int lds_bytes, unsigned* ctr, unsigned* err,
                       unsigned long long timeout_ticks, hipStream_t s) {
  if (lds_bytes < 4) lds_bytes = 4;
  static const bool attr = [] {
    raise_dyn_lds((const void*)fanin_probe_kernel);
    return true;
  }();
  (void)attr;
  DPPO_LAUNCH(fanin_probe_kernel, dim3((unsigned)blocks), dim3(1024), (size_t)lds_bytes, s, ctr,
              err, timeout_ticks);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_clip_adam(float* params, float* grad, float* m, float* v, int64_t n, float max_norm,
                     float neg_step_size, float bc2_sqrt, float beta1, float beta2, float eps,
                     float* out_norm, hipStream_t s) {
  return launch_clip_adam_traced(params, grad, m, v, n, nullptr, 0, max_norm, neg_step_size,
                                 bc2_sqrt, beta1, beta2, eps, out_norm, nullptr, 0.f, 0.f, 0.f, s);
}

}  // namespace dppo
