// GAE, advantage statistics / normalisation, and sample-record packing for gfx950.
//
// GAE replaces PPO.calculate_advantage (reference diamond/ppo.py:188-222; identical code in
// continuous_ppo.py:200-234 and recurrent_ppo.py:265-299) fused with returns = values + adv
// (ppo.py:241) and the per-tile partial sums for the normalisation (ppo.py:243).
//
// Roofline: HBM-bound, 22 algorithmic bytes per element (rewards, values, next_values 4 B each,
// term/trunc 1 B each read; advantages and returns 4 B each written), ~0.5 FLOP/B.
//
// The recurrence is serial per env (bit-exactness forbids re-association) but only 2 dependent
// flops per step; the bytes are what cost.  gae_pipe_kernel (below) overlaps the loads, the scan
// and the stores of one env tile; gae_kernel is the plain stage-all / scan / store-all form, kept
// for unaligned shapes (N not a multiple of 16 or unaligned buffers).
#include <cstdlib>

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

// ---- Pipelined GAE (aligned shapes: the one learn() and the benchmark use) ---------------------
// Persistent: at most one workgroup per CU, walking env tiles of E envs -- E = 32 (each row of a
// [T][N] float buffer one 128-B line) when that still gives every CU a tile, else E = 16; tiles
// that share 128-B lines run on one XCD (pipe_tile).  The serial recurrence is the latency floor,
// so a workgroup scans ALL its envs in one pass: lanes are free, the 128 dependent steps are not.
// 9 waves per workgroup:
//  * waves 0..7 each own one 16-step chunk of the current 128-step super-chunk (wave w chunk
//    7 - w: waves issue roughly in wave order, so the chunk the scan needs first is requested
//    first; measured 0.4-0.6 us better than wave w -> chunk w at N = 8192).  An owner loads
//    its chunk (16-B loads along the env axis), computes every term of the recurrence that does
//    not depend on the carried advantage -- delta = (r + (gamma*nv)*nt) - v and
//    coef = (c*nt)*ntr, the reference's op order -- and writes them env-major into LDS, flags the
//    chunk, waits until the scan has passed it, then stores advantages and returns = v + a
//    (16-B stores) and accumulates the normalisation statistics;
//  * wave 8 is the scan (lane = env): per chunk 8 ds_read_b128, then 16 dependent steps of
//    a = delta + coef * a (two VALU ops each), 4 ds_write_b128; fully unrolled over the 8 chunks
//    with the operands of the next two chunks already requested, so the chain waits only for
//    reads issued two chunks earlier (the rolled loop's loop-carried register copies made every
//    chunk wait for the next chunk's prefetch: 1.2 us; one chunk of look-ahead still exposed the
//    LDS latency under the owners' traffic: ~650 cycles per chunk).
// Timing-only builds: DPPO_GAE_TRACE (hand-off timeline, tools/gae_trace.py), DPPO_GAE_NOSCAN
// (no recurrence: the movement-only time of this structure, wrong results).
// An owner that has stored its chunk of tile i goes straight on to its chunk of tile i + 1, so
// the chunks the scan reaches first (latest in time) start loading the next tile while the
// scan is still walking back through the current one: loads and stores of different tiles
// overlap.  Bit-exact with gae_step (same fp32 operations, FMA contraction off).
constexpr int kPChunk = 16;
constexpr int kPChunks = 8;
constexpr int kPSuper = kPChunk * kPChunks;
constexpr int kPThreads = (kPChunks + 1) * kWave;
constexpr int kPStride = kPSuper + 4;

#ifdef DPPO_GAE_TRACE
// Timing-only build: workgroups 0 and 128 stamp s_memtime at the pipeline's hand-off points.
// [wg][slot]: 0 start; 1+k owner k loads landed; 9+k owner k scan-wait done; 17+k owner k stores
// issued; 25+k scanner chunk k flag seen; 33+k scanner chunk k done; 41 end.
__device__ long long g_gae_trace[2][48];
#define GAE_STAMP(slot)                                                                  \
  do {                                                                                  \
    if ((blockIdx.x == 0 || blockIdx.x == 128) && (threadIdx.x & 63) == 0 &&           \
        (slot != 0 || threadIdx.x == 0) && (slot != 41 || threadIdx.x == 0))          \
      g_gae_trace[blockIdx.x ? 1 : 0][slot] = __builtin_amdgcn_s_memtime();            \
  } while (0)
// the "loads landed" stamps (1 + k) first wait for the chunk's loads and LDS writes: s_memtime has
// no data dependency, so without the wait it can issue before the data it is meant to time
#define GAE_STAMP_LANDED(slot)                                      \
  do {                                                              \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");     \
    GAE_STAMP(slot);                                                \
  } while (0)
#else
#define GAE_STAMP(slot) \
  do {                  \
  } while (0)
#define GAE_STAMP_LANDED(slot) \
  do {                         \
  } while (0)
#endif // env-major rows: 16-B aligned, conflict-free b128 reads

template <int E>
struct PipeLds {
  float delta[E][kPStride];
  float coef[E][kPStride];
  float a[E][kPStride];
  double wsum[kPChunks][2];
  int loaded[kPChunks];
  int scanned[kPChunks];
};

// LDS row swizzle of the env-major operand rows (DPPO_GAE_SWZ builds only): element (env, t) of a
// super-chunk at column t ^ 12 (env >> 4 & 3).  Rows are 132 floats apart (16-B aligned for the
// scan's ds_read_b128), so the owners' 4-B writes -- lane (env 4m + j, row) -- land 4 lanes per
// bank at 64-env tiles and 2 at 32.  The swizzle keeps every 4-row group contiguous and aligned
// and the scan's reads conflict-free; measured (round 5, rocprofv3, 2 reps): bank-conflict share
// at N = 65,536 62.3 % -> 35.8 %, but the launch 39.3 -> 41.0-43.2 us (the per-access XOR on the
// owners' and the scan's addresses), and 8.0 -> 8.05-8.1 us at 8,192.  The conflicts are not on
// the launch's critical path (it waits on the arrival of the loads, §3.2): off by default.
__device__ __forceinline__ int pswz(int env) {
#ifdef DPPO_GAE_SWZ
  return 12 * ((env >> 4) & 3);
#else
  return 0 * env;
#endif
}

__device__ __forceinline__ void gae_terms(float r, float v, float nv, float te, float tr, float g,
                                          float c, float& delta, float& coef) {
#pragma clang fp contract(off)
  const float nt = 1.0f - te;                 // ppo.py:202-203
  const float ntr = 1.0f - tr;
  delta = (r + (g * nv) * nt) - v;            // ppo.py:206-210
  coef = (c * nt) * ntr;                      // ppo.py:214-218
}

// 16-B store written through to memory (sc1): the line leaves the XCD's L2 while the kernel runs
// instead of as a dirty line written back at the kernel boundary (MI355X_MICROARCH.md
// publish-large / boundary: a predecessor leaving B dirty bytes costs ~B / 6 TB/s)
__device__ __forceinline__ void store_wt(float* p, f32x4 v) {
  // s_nop: a VALU write to the data VGPRs of a store wider than 8 bytes needs a wait state
  // after it, which the compiler cannot insert behind an asm statement (seen: back-to-back slab
  // stores whose next operands overwrote this one's data before it was read)
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ float gae_carry(float delta, float coef, float a) {
#pragma clang fp contract(off)
  return delta + coef * a;                    // ppo.py:213-219
}

// The normalisation statistics (ppo.py:243) of a row's 4 advantages, in fp32 and in a fixed
// order, shifted by the lane's first advantage of the chunk (sft): the caller adds one fp32
// partial per chunk (<= 8 values) into its fp64 sums as sum x = S + n sft and
// sum x^2 = Q + sft (2 S + n sft).  Per-value fp64 accumulation cost 3 half-rate fp64 operations
// per value on the SIMD the scan runs on; unshifted fp32 partials lose the variance when the
// advantages' mean dwarfs their spread (std off by 1.6e-5 at mean / std = 1,000; shifted 7e-9).
__device__ __forceinline__ void stats4(const f32x4& av, float sft, float& s, float& q) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float dx = av[j] - sft;
    s += dx;
    q = __builtin_fmaf(dx, dx, q);
  }
}

__device__ __forceinline__ void stats_fold(float s32, float q32, float sft, int cnt, double& lsum,
                                           double& lsq) {
  const double ds = (double)sft, dn = (double)cnt, dsum = (double)s32;
  lsum += dsum + dn * ds;
  lsq += (double)q32 + ds * (2.0 * dsum + dn * ds);
}

__device__ __forceinline__ void wait_flag(int* f, int gen) {
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < gen)
    __builtin_amdgcn_s_sleep(1);
}

// Publish LDS data to the other waves of the workgroup: a wave's LDS operations are performed in
// program order, so a flag store issued after the data stores is seen after them by any wave that
// reads the flag and then the data -- no s_waitcnt lgkmcnt(0) (what a release would emit) in
// front of it; only the compiler must keep the order (signal fence).  DPPO_GAE_RELEASE: the
// release store (A/B timing).
__device__ __forceinline__ void set_flag(int* f, int gen) {
#ifdef DPPO_GAE_RELEASE
  __hip_atomic_store(f, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __hip_atomic_store(f, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}

// logical tile lb -> env tile, XCD-aware (speed only): the K = 128 / E tiles whose flag bytes
// share one 128-B line of term / trunc (and, for E = 16, whose floats share lines pairwise) go to
// blocks lb, lb + 8, lb + 16, ... -- one XCD under round-robin dispatch, so the line is fetched
// into one L2 once instead of into K different XCDs' L2s (measured before: 4x the flag bytes,
// 21 MB read per launch at N = 8192 for 14.7 MB of operands)
template <int E>
__device__ __forceinline__ int pipe_tile(int lb, int ntiles) {
  constexpr int K = 128 / E, G = 8 * K;
  const int grp = lb / G, r = lb % G;
  return (grp + 1) * G <= ntiles ? grp * G + K * (r & 7) + (r >> 3) : lb;
}

// The streaming variants of the owners' global accesses and the tile map (NT bits, A/B via
// DPPO_GAE_NT; tools/probe/stream_probe2.hip measured each on the launch's bare data movement):
//   1 non-temporal operand loads, 2 non-temporal advantage / return stores,
//   4 XCD-contiguous tiles: the blocks one XCD runs (round-robin dispatch) take one contiguous
//     eighth of the env axis (groups of K = 128 / E tiles sharing a flag line stay on one XCD)
template <int NT, typename T>
__device__ __forceinline__ T gld(const T* p) {
  if (NT & 1) return __builtin_nontemporal_load(p);
  return *p;
}
template <int NT, typename T>
__device__ __forceinline__ void gst(T* p, T v) {
  if (NT & 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <int E, int NT>
__device__ __forceinline__ int pipe_tile_nt(int lb, int ntiles) {
  constexpr int K = 128 / E;
  if ((NT & 4) && ntiles % (8 * K) == 0) return (lb % 8) * (ntiles / 8) + lb / 8;
  return pipe_tile<E>(lb, ntiles);
}

template <int E, int NT = 0>
__global__ __launch_bounds__(kPThreads) void gae_pipe_kernel(
    const float* __restrict__ rew, const uint8_t* __restrict__ term,
    const uint8_t* __restrict__ trunc, const float* __restrict__ val,
    const float* __restrict__ nval, float* __restrict__ adv, float* __restrict__ ret,
    double* __restrict__ partials, int T, int N, float g, float c, int wt, int stagger,
    int psleep) {
  __shared__ __attribute__((aligned(16))) PipeLds<E> L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntiles = N / E;
  const int nsup = (T + kPSuper - 1) / kPSuper;
  if (threadIdx.x < kPChunks) {
    L.loaded[threadIdx.x] = 0;
    L.scanned[threadIdx.x] = 0;
  }
  __syncthreads();
  GAE_STAMP(0);
  if (wave < kPChunks) {
    // ---------------- chunk owner
    constexpr int V4 = E / 4;              // lanes per row (4 envs each)
    constexpr int RP = kWave / V4;         // rows per pass
    constexpr int PER = kPChunk / RP;      // passes per chunk (2 for E = 32, 1 for E = 16)
    // wave w owns chunk 7 - w: waves issue roughly in wave order, so the chunk the scan needs
    // first (latest in time) is requested first and tends to land first
    const int k = kPChunks - 1 - wave;
    const int e0 = 4 * (lane % V4);
    const int sw = pswz(e0);  // the same for e0 .. e0 + 3
    double lsum = 0.0, lsq = 0.0;
    int gen = 0;
    // Staggered start of the first tile's loads: owner w (chunk 7 - w) issues `stagger` cycles
    // after owner w - 1, so the chunks arrive in the order the scan consumes them instead of all
    // together at the end of the chip-wide read burst, and the scan starts under the burst.
    if (stagger > 0 && wave > 0) {
      const long long until = (long long)__builtin_amdgcn_s_memtime() + (long long)wave * stagger;
      while ((long long)__builtin_amdgcn_s_memtime() < until) __builtin_amdgcn_s_sleep(2);
    }
    for (int lb = blockIdx.x; lb < ntiles; lb += gridDim.x) {
      const int n0 = pipe_tile_nt<E, NT>(lb, ntiles) * E;
      for (int s = 0; s < nsup; ++s) {
        ++gen;
        const int hi = T - s * kPSuper;
        const int lo = hi > kPSuper ? hi - kPSuper : 0;
        const int r0 = k * kPChunk;
        const int nr = min(kPChunk, hi - lo - r0);
        // (nr <= 0: no such chunk in this super-chunk -- it is written as identity rows, so the
        // scan always walks all kPChunks chunks and can be fully unrolled)
        f32x4 xr[PER], xv[PER], xn[PER];
        uint32_t xt[PER], xu[PER];
#pragma unroll
        for (int p = 0; p < PER; ++p) {  // every load of the chunk in flight at once
          const int row = p * RP + lane / V4;
          if (row < nr) {
            const int64_t go = (int64_t)(lo + r0 + row) * N + n0 + e0;
            // (NT & 8: non-temporal loads of the rollout's own inputs only -- rewards and
            // flags, staged long before -- and plain ones of the values the eval kernel has
            // just written)
            constexpr int NTI = (NT & 8) ? (NT | 1) : NT;
            xr[p] = gld<NTI>((const f32x4*)(rew + go));
            xv[p] = gld<NT>((const f32x4*)(val + go));
            xn[p] = gld<NT>((const f32x4*)(nval + go));
            xt[p] = gld<NTI>((const uint32_t*)(term + go));
            xu[p] = gld<NTI>((const uint32_t*)(trunc + go));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < PER; ++p) {
          const int row = p * RP + lane / V4;
          if (row < nr) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float d, cf;
              gae_terms(xr[p][j], xv[p][j], xn[p][j], ((xt[p] >> (8 * j)) & 0xffu) ? 1.0f : 0.0f,
                        ((xu[p] >> (8 * j)) & 0xffu) ? 1.0f : 0.0f, g, c, d, cf);
              L.delta[e0 + j][(r0 + row) ^ sw] = d;
              L.coef[e0 + j][(r0 + row) ^ sw] = cf;
            }
          } else {
            // rows past the end of the rollout: a = -0 + 1 * a is the identity for every a
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              L.delta[e0 + j][(r0 + row) ^ sw] = -0.0f;
              L.coef[e0 + j][(r0 + row) ^ sw] = 1.0f;
            }
          }
        }
        if (lane == 0) set_flag(&L.loaded[k], gen);
        GAE_STAMP_LANDED(1 + k);
        wait_flag(&L.scanned[k], gen);
        GAE_STAMP(9 + k);
        float s32 = 0.0f, q32 = 0.0f, sft = 0.0f;
        int cnt = 0;
        // every pass's advantages read before the first store: the write-through stores are asm
        // with a memory clobber, so reads placed after one wait for their own LDS round trip
        f32x4 avp[PER];
#pragma unroll
        for (int p = 0; p < PER; ++p) {
          const int row = p * RP + lane / V4;
          if (row < nr) {
#pragma unroll
            for (int j = 0; j < 4; ++j) avp[p][j] = L.a[e0 + j][(r0 + row) ^ sw];
          }
        }
#pragma unroll
        for (int p = 0; p < PER; ++p) {
          const int row = p * RP + lane / V4;
          if (row < nr) {
            const int64_t go = (int64_t)(lo + r0 + row) * N + n0 + e0;
            const f32x4 av = avp[p];
            if (p == 0) sft = av[0];  // (a later pass has a row only if pass 0 has one)
            if (wt) {
              store_wt(adv + go, av);
              store_wt(ret + go, xv[p] + av);  // returns = values + advantages (ppo.py:241)
            } else {
              gst<NT>((f32x4*)(adv + go), av);
              gst<NT>((f32x4*)(ret + go), xv[p] + av);
            }
            stats4(av, sft, s32, q32);
            cnt += 4;
          }
        }
        stats_fold(s32, q32, sft, cnt, lsum, lsq);
        GAE_STAMP(17 + k);
      }
    }
    // this wave's statistics partial (fixed order)
    lsum = wave_sum_f64(lsum);
    lsq = wave_sum_f64(lsq);
    if (lane == 0) {
      L.wsum[k][0] = lsum;
      L.wsum[k][1] = lsq;
    }
  } else if (lane < E) {
    // ---------------- the scan, one lane per env, all kPChunks chunks of every super-chunk
    // (missing ones are identity rows), fully unrolled over three static operand register sets:
    // while chunk k's 16 dependent steps run, chunk k-1's operands are already in registers and
    // chunk k-2's LDS reads are in flight -- the chain never waits for reads issued during the
    // previous chunk (with one chunk of look-ahead it did: ~650 cycles per 16-step chunk under
    // the owners' LDS traffic, against ~250 now).
    const int e = lane;
    const int sw = pswz(e);
    int gen = 0;
    // The scan is the youngest wave of the workgroup and shares its SIMD with two owners: at the
    // default priority every owner VALU instruction issues first (age order) and the dependent
    // chain crawls at ~30 cycles per step.  It is the critical path: give it the SIMD.
    // (psleep & 4, A/B: raise it only once the first chunk has been seen, so that the owners on
    // this SIMD issue their first loads at normal priority)
    if (!(psleep & 4)) __builtin_amdgcn_s_setprio(3);
    for (int lb = blockIdx.x; lb < ntiles; lb += gridDim.x) {
      float a = 0.0f;  // advantage carried backwards, 0 after the last step (ppo.py:198)
      for (int s = 0; s < nsup; ++s) {
        ++gen;
        f32x4 d[3][4], cf[3][4];
        int pf[kPChunks];  // the chunk flag seen just before its speculative prefetch
        auto fetch = [&](int k, int set) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            d[set][q] = *(const f32x4*)&L.delta[e][(k * kPChunk + 4 * q) ^ sw];
            cf[set][q] = *(const f32x4*)&L.coef[e][(k * kPChunk + 4 * q) ^ sw];
          }
        };
        // Wait for chunk k by polling its flag and its data together: the flag read is performed
        // before the data reads (one wave's LDS operations complete in order), so the poll that
        // sees the flag set already holds current data -- one LDS round trip after the owner's
        // flag store instead of two (poll the flag, then fetch).
        auto poll = [&](int k, int set) {
          int f;
          do {
            f = __hip_atomic_load(&L.loaded[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            __builtin_amdgcn_sched_barrier(0);
            fetch(k, set);
            // keep every poll's data reads in the loop (without a use, the compiler sinks them
            // behind it: flag round trip, then data round trip)
#pragma unroll
            for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(d[set][q]), "+v"(cf[set][q]));
            if (f >= gen) break;
            // (psleep: back off between unsuccessful polls -- each poll is 9 LDS reads, which
            // otherwise compete with the owners' term writes for the LDS)
            if ((psleep & 3) == 1) __builtin_amdgcn_s_sleep(1);
            else if ((psleep & 3) >= 2) __builtin_amdgcn_s_sleep(2);
          } while (true);
        };
        poll(kPChunks - 1, (kPChunks - 1) % 3);
        if (psleep & 4) __builtin_amdgcn_s_setprio(3);
        pf[kPChunks - 1] = gen;
        // speculative prefetch of chunk k-1 / k-2: its flag is read before its data (LDS
        // operations of one wave complete in order), so a set flag proves the data current
        pf[kPChunks - 2] =
            __hip_atomic_load(&L.loaded[kPChunks - 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __builtin_amdgcn_sched_barrier(0);
        fetch(kPChunks - 2, (kPChunks - 2) % 3);
#pragma unroll
        for (int k = kPChunks - 1; k >= 0; --k) {
          const int b = k % 3;
          GAE_STAMP(25 + k);
          if (k >= 2) {
            pf[k - 2] = __hip_atomic_load(&L.loaded[k - 2], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_sched_barrier(0);
            fetch(k - 2, (k - 2) % 3);
          }
          // The 16 dependent steps, in both arms of the re-read test: with one copy after the
          // join, the join's wait had to cover the re-read arm's loads (s_waitcnt lgkmcnt(0)), so
          // the fast arm also waited for chunk k-2's prefetch, issued just above -- one LDS round
          // trip under the owners' traffic exposed in front of every chunk.
          auto chain = [&]() {
#ifndef DPPO_GAE_NOSCAN
            f32x4 av[4];
#pragma unroll
            for (int j = kPChunk - 1; j >= 0; --j) {
              a = gae_carry(d[b][j >> 2][j & 3], cf[b][j >> 2][j & 3], a);
              av[j >> 2][j & 3] = a;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) *(f32x4*)&L.a[e][(k * kPChunk + 4 * q) ^ sw] = av[q];
#endif
          };
          if (pf[k] < gen) {  // prefetched before its owner published it: poll and re-read
            poll(k, b);
            chain();
          } else {
            chain();
          }
          if (lane == 0) set_flag(&L.scanned[k], gen);
          GAE_STAMP(33 + k);
        }
      }
    }
  }
  __syncthreads();
  GAE_STAMP(41);
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0;
    for (int k = 0; k < kPChunks; ++k) {
      s0 += L.wsum[k][0];
      s1 += L.wsum[k][1];
    }
    partials[2 * blockIdx.x] = s0;
    partials[2 * blockIdx.x + 1] = s1;
  }
}

// ---- Affine-scan GAE (tolerance mode, SURVEY §7.2 hard part 1 / §8(c): <= 1e-6 relative) ------
// The recurrence a_t = delta_t + coef_t * a_{t+1} is an affine map of the carried advantage, and
// affine maps compose: over a 16-step chunk, a_j = b_j + p_j * a_end with b, p the chunk's local
// scan from the identity (b = 0, p = 1 at its end).  So every chunk owner scans its own 16 steps
// at once -- all 8 owners of a 128-step super-chunk in parallel, instead of one wave walking 128
// dependent steps -- and publishes its chunk map (B, P) = (b_0, p_0) in LDS with a per-chunk flag.
// The owner of chunk k then waits ONLY for the maps of the later chunks j > k (no workgroup
// barrier), folds them into the super-chunk's carry in the fixed order j = 7 .. k + 1 (<= 7
// dependent steps: the same operations, so the same bits, whatever the arrival order), finishes
// its 16 advantages and stores them at once -- stores leave chunk by chunk as the loads land.
// The owners start their first loads staggered (wave w = chunk 7 - w, `stagger` cycles apart), as
// in gae_pipe_kernel, so chunks land in the order the folds need them.  The chunk that ends the
// rollout is bit-exact (carry 0); elsewhere the re-association costs a few ulp (the parity test
// bounds it at 1e-6 of the advantages' scale).
// Buffers reused across iterations (tile, super-chunk) are double-buffered by iteration parity,
// with back-pressure where a writer could lap a reader: the owner of chunk k rewrites its map
// slot only after every lower chunk's owner has read the map it holds (rdone), and the carry
// slot (written by chunk 0's owner) is only rewritten after every owner published its next map.
// DPPO_GAE_AFF_BARRIER: the round-3 form (one workgroup barrier per iteration; A/B timing).
template <int E>
struct AffLds {
  float delta[E][kPStride];  // env-major rows of this super-chunk (wave-private row ranges)
  float coef[E][kPStride];
  float a[E][kPStride];
  float B[2][kPChunks][E];   // chunk maps, double-buffered by iteration parity
  float P[2][kPChunks][E];
  float carry[2][E];         // advantage at the start of the previous super-chunk
  int mflag[kPChunks];       // iteration (gen) whose map chunk k's slot holds
  int rdone[kPChunks];       // last iteration whose later-chunk maps chunk k's owner has read
  int cflag;                 // last iteration whose carry-out chunk 0's owner has published
  double wsum[kPChunks][2];
};

__device__ __forceinline__ int lds_ld(const int* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// After a poll loop on LDS flags: keep the compiler from moving the LDS accesses that the flags
// guard above the loop (the hardware performs one wave's LDS operations in order)
__device__ __forceinline__ void after_poll() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }

template <int E>
__global__ __launch_bounds__(kPChunks * kWave) void gae_aff_kernel(
    const float* __restrict__ rew, const uint8_t* __restrict__ term,
    const uint8_t* __restrict__ trunc, const float* __restrict__ val,
    const float* __restrict__ nval, float* __restrict__ adv, float* __restrict__ ret,
    double* __restrict__ partials, int T, int N, float g, float c, int stagger) {
  __shared__ __attribute__((aligned(16))) AffLds<E> L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int k = kPChunks - 1 - wave;     // wave w owns chunk 7 - w (the latest chunk loads first)
  const int ntiles = N / E;
  const int nsup = (T + kPSuper - 1) / kPSuper;
  constexpr int V4 = E / 4;              // lanes per row (4 envs each)
  constexpr int RP = kWave / V4;         // rows per pass
  constexpr int PER = kPChunk / RP;      // passes per chunk
  const int e0 = 4 * (lane % V4);
  const int r0 = k * kPChunk;
  if (threadIdx.x < kPChunks) {
    L.mflag[threadIdx.x] = 0;
    L.rdone[threadIdx.x] = 0;
  }
  if (threadIdx.x == 0) L.cflag = 0;
  __syncthreads();
  // iterations q = (tile, super-chunk) pairs of this workgroup, super-chunks latest first
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int niter = my_tiles * nsup;
  struct Ops {
    f32x4 r[PER], v[PER], nv[PER];
    uint32_t te[PER], tr[PER];
  };
  auto geom = [&](int q, int64_t& base, int& lo, int& nr, int& s) {
    const int lb = blockIdx.x + (q / nsup) * gridDim.x;
    s = q % nsup;
    const int hi = T - s * kPSuper;
    lo = hi > kPSuper ? hi - kPSuper : 0;
    nr = min(kPChunk, hi - lo - r0);
    base = (int64_t)(lo + r0) * N + pipe_tile<E>(lb, ntiles) * E + e0;
  };
  auto load = [&](int q, Ops& o) {
    int64_t base;
    int lo, nr, s;
    geom(q, base, lo, nr, s);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int row = p * RP + lane / V4;
      if (row < nr) {
        const int64_t go = base + (int64_t)row * N;
        o.r[p] = *(const f32x4*)(rew + go);
        o.v[p] = *(const f32x4*)(val + go);
        o.nv[p] = *(const f32x4*)(nval + go);
        o.te[p] = *(const uint32_t*)(term + go);
        o.tr[p] = *(const uint32_t*)(trunc + go);
      }
    }
  };
  double lsum = 0.0, lsq = 0.0;
  GAE_STAMP(0);
  if (stagger > 0 && wave > 0) {
    const long long until = (long long)__builtin_amdgcn_s_memtime() + (long long)wave * stagger;
    while ((long long)__builtin_amdgcn_s_memtime() < until) __builtin_amdgcn_s_sleep(2);
  }
  Ops cur{}, nxt{};
  if (niter > 0) load(0, cur);
  for (int q = 0; q < niter; ++q) {
    const int par = q & 1, gen = q + 1;
    int64_t base;
    int lo, nr, s;
    geom(q, base, lo, nr, s);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int row = p * RP + lane / V4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d = -0.0f, cf = 1.0f;  // rows past the rollout: the identity map
        if (row < nr)
          gae_terms(cur.r[p][j], cur.v[p][j], cur.nv[p][j],
                    ((cur.te[p] >> (8 * j)) & 0xffu) ? 1.0f : 0.0f,
                    ((cur.tr[p] >> (8 * j)) & 0xffu) ? 1.0f : 0.0f, g, c, d, cf);
        L.delta[e0 + j][r0 + row] = d;
        L.coef[e0 + j][r0 + row] = cf;
      }
    }
    GAE_STAMP_LANDED(1 + k);
    // the next iteration's operands go out now: they land while this one is scanned and stored
    if (q + 1 < niter) load(q + 1, nxt);
    // local scan of the chunk from the identity, lane = env (this wave's own LDS rows: its LDS
    // operations complete in order)
    float bl[kPChunk], pl[kPChunk];
    float cin = 0.0f;
    if (lane < E) {
      f32x4 d4[4], c4[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        d4[qq] = *(const f32x4*)&L.delta[lane][r0 + 4 * qq];
        c4[qq] = *(const f32x4*)&L.coef[lane][r0 + 4 * qq];
      }
      float b = 0.0f, pp = 1.0f;
#pragma unroll
      for (int j = kPChunk - 1; j >= 0; --j) {
        b = gae_carry(d4[j >> 2][j & 3], c4[j >> 2][j & 3], b);
        pp = c4[j >> 2][j & 3] * pp;
        bl[j] = b;
        pl[j] = pp;
      }
    }
#ifdef DPPO_GAE_AFF_BARRIER
    if (lane < E) {
      L.B[par][k][lane] = bl[0];
      L.P[par][k][lane] = pl[0];
    }
    GAE_STAMP(9 + k);
    __syncthreads();
    GAE_STAMP(25 + k);
    if (lane < E) {
      cin = s == 0 ? 0.0f : L.carry[par][lane];
      float Bj[kPChunks], Pj[kPChunks];
#pragma unroll
      for (int j = 0; j < kPChunks; ++j) {
        Bj[j] = L.B[par][j][lane];
        Pj[j] = L.P[par][j][lane];
      }
#pragma unroll
      for (int j = kPChunks - 1; j > 0; --j)
        if (j > k) cin = gae_carry(Bj[j], Pj[j], cin);
    }
#else
    // back-pressure: this map slot was last written for iteration q - 2; every lower chunk's
    // owner must have read it (rdone) before it is overwritten
    if (gen > 2) {
      bool ok;
      do {
        ok = true;
#pragma unroll
        for (int j = 0; j < kPChunks; ++j)
          if (j < k && lds_ld(&L.rdone[j]) < gen - 2) ok = false;
        if (!ok) __builtin_amdgcn_s_sleep(1);
      } while (!ok);
      after_poll();
    }
    if (lane < E) {
      L.B[par][k][lane] = bl[0];
      L.P[par][k][lane] = pl[0];
    }
    if (lane == 0) set_flag(&L.mflag[k], gen);
    GAE_STAMP(9 + k);
    // the carry into the super-chunk (chunk 0's owner published it one iteration earlier)
    if (s > 0) {
      while (lds_ld(&L.cflag) < gen - 1) __builtin_amdgcn_s_sleep(1);
      after_poll();
    }
    // the later chunks' maps: poll their flags, then read every map at once
    {
      bool ok;
      do {
        ok = true;
#pragma unroll
        for (int j = 0; j < kPChunks; ++j)
          if (j > k && lds_ld(&L.mflag[j]) < gen) ok = false;
        if (!ok) __builtin_amdgcn_s_sleep(1);
      } while (!ok);
      after_poll();
    }
    GAE_STAMP(25 + k);
    if (lane < E) {
      cin = s == 0 ? 0.0f : L.carry[par][lane];
      float Bj[kPChunks], Pj[kPChunks];
#pragma unroll
      for (int j = 0; j < kPChunks; ++j) {
        Bj[j] = j > k ? L.B[par][j][lane] : 0.0f;
        Pj[j] = j > k ? L.P[par][j][lane] : 1.0f;
      }
      // the fold in the fixed order j = 7 .. k + 1: the same bits whatever the arrival order
#pragma unroll
      for (int j = kPChunks - 1; j > 0; --j)
        if (j > k) cin = gae_carry(Bj[j], Pj[j], cin);
    }
    if (lane == 0) set_flag(&L.rdone[k], gen);   // (LDS operations of a wave complete in order)
#endif
    if (lane < E) {
      f32x4 av[4];
#pragma unroll
      for (int j = 0; j < kPChunk; ++j) av[j >> 2][j & 3] = gae_carry(bl[j], pl[j], cin);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) *(f32x4*)&L.a[lane][r0 + 4 * qq] = av[qq];
      if (k == 0) L.carry[par ^ 1][lane] = av[0][0];  // for the super-chunk before this one
    }
#ifndef DPPO_GAE_AFF_BARRIER
    if (k == 0 && lane == 0) set_flag(&L.cflag, gen);
#endif
    GAE_STAMP(33 + k);
    float s32 = 0.0f, q32 = 0.0f, sft = 0.0f;
    int cnt = 0;
    f32x4 avp[PER];
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int row = p * RP + lane / V4;
      if (row < nr) {
#pragma unroll
        for (int j = 0; j < 4; ++j) avp[p][j] = L.a[e0 + j][r0 + row];
      }
    }
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int row = p * RP + lane / V4;
      if (row < nr) {
        const int64_t go = base + (int64_t)row * N;
        const f32x4 av = avp[p];
        *(f32x4*)(adv + go) = av;
        *(f32x4*)(ret + go) = cur.v[p] + av;  // returns = values + advantages (ppo.py:241)
        if (p == 0) sft = av[0];
        stats4(av, sft, s32, q32);
        cnt += 4;
      }
    }
    stats_fold(s32, q32, sft, cnt, lsum, lsq);
    GAE_STAMP(17 + k);
    cur = nxt;
  }
  lsum = wave_sum_f64(lsum);
  lsq = wave_sum_f64(lsq);
  if (lane == 0) {
    L.wsum[k][0] = lsum;
    L.wsum[k][1] = lsq;
  }
  __syncthreads();
  GAE_STAMP(41);
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0;
    for (int j = 0; j < kPChunks; ++j) {
      s0 += L.wsum[j][0];
      s1 += L.wsum[j][1];
    }
    partials[2 * blockIdx.x] = s0;
    partials[2 * blockIdx.x + 1] = s1;
  }
}

// Sum the per-tile partials in a fixed order (256 threads): {sum, sumsq} in s0[0], s1[0].
__device__ __forceinline__ void partials_sum256(const double* __restrict__ partials, int n,
                                                double* s0, double* s1) {
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
}

// dsum = {sum, sumsq} of the per-tile partials.
__global__ __launch_bounds__(256) void stats_reduce_kernel(const double* __restrict__ partials,
                                                           int n, double* __restrict__ dsum) {
  __shared__ double s0[256], s1[256];
  partials_sum256(partials, n, s0, s1);
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
// A block packs 256 consecutive samples through LDS: the [256][D] observation rows and the
// [256][A] continuous actions are read as one contiguous run each, the [256][R] records are
// assembled in LDS and leave as one contiguous run of 16-B stores (a record is R = 12..52 floats:
// storing it per thread scattered 16-B pieces over every line and doubled the written bytes).
constexpr int kPackTile = 256;

static_assert(kPackTile == 256, "pack_kernel reduces the statistics with 256 threads");
__global__ __launch_bounds__(kPackTile) void pack_kernel(PackArgs a) {
  extern __shared__ __attribute__((aligned(16))) float pk_lds[];
  float* obs_s = pk_lds;                          // [256][D]
  float* act_s = obs_s + kPackTile * a.D;         // [256][A] (continuous)
  float* rec_s = act_s + (a.continuous ? kPackTile * a.A : 0);  // [256][R], 16-B aligned rows
  float mean = 0.0f, denom = 1.0f;
  if (a.advantage_norm) {
    float sd;
    if (a.partials) {
      // the statistics launch folded in: every block reduces the GAE partials itself, in
      // stats_reduce_kernel's order (the same bits in every block and as the separate launch)
      __shared__ double s0[kPackTile], s1[kPackTile];
      partials_sum256(a.partials, a.n_partials, s0, s1);
      const double ds[2] = {s0[0], s1[0]};
      mean_std_from(ds, a.n_total, &mean, &sd);
    } else {
      mean_std_from(a.dsum, a.n_total, &mean, &sd);
    }
    denom = sd + 1e-6f;
  }
  const int t = threadIdx.x;
  for (int64_t i0 = (int64_t)blockIdx.x * kPackTile; i0 < a.B;
       i0 += (int64_t)gridDim.x * kPackTile) {
    const int ns = (int)min((int64_t)kPackTile, a.B - i0);
    const float* o = a.obs + i0 * a.D;
    // observation rows of a multiple of 4 features: 16-B loads and 16-B LDS accesses (the 4-B
    // per-feature form put a row stride of D floats across the lanes: 8-way LDS bank conflicts at
    // D = 8, 64 % of the kernel's LDS cycles)
    const bool q4 = (a.D & 3) == 0 && ((uintptr_t)a.obs & 15) == 0;
    if (q4) {
      const f32x4* o4 = (const f32x4*)o;
      for (int e = t; e < ns * a.D / 4; e += kPackTile) ((f32x4*)obs_s)[e] = o4[e];
    } else if (((uintptr_t)a.obs & 15) == 0) {
      // other widths: the tile's block of ns * D floats starts 16-B aligned (i0 is a multiple of
      // 256), so it still moves as 16-B pieces plus a scalar tail
      const int n4 = ns * a.D / 4;
      for (int e = t; e < n4; e += kPackTile) ((f32x4*)obs_s)[e] = ((const f32x4*)o)[e];
      for (int e = 4 * n4 + t; e < ns * a.D; e += kPackTile) obs_s[e] = o[e];
    } else {
      for (int e = t; e < ns * a.D; e += kPackTile) obs_s[e] = o[e];
    }
    if (a.continuous) {
      const float* ac = (const float*)a.actions + i0 * a.A;
      if (((uintptr_t)a.actions & 15) == 0) {
        const int n4 = ns * a.A / 4;
        for (int e = t; e < n4; e += kPackTile) ((f32x4*)act_s)[e] = ((const f32x4*)ac)[e];
        for (int e = 4 * n4 + t; e < ns * a.A; e += kPackTile) act_s[e] = ac[e];
      } else {
        for (int e = t; e < ns * a.A; e += kPackTile) act_s[e] = ac[e];
      }
    }
    __syncthreads();
    if (t < ns) {
      const int64_t i = i0 + t;
      float* r = rec_s + t * a.R;
      if (q4) {
        // the record's observation part as 16-B moves (a record row is R = 12..52 floats, 16-B
        // aligned: lanes 48+ B apart touch distinct banks within each 8-lane group)
        const f32x4* src = (const f32x4*)(obs_s + t * a.D);
        for (int k = 0; k < a.D8 / 4; ++k)
          ((f32x4*)r)[k] = 4 * k < a.D ? src[k] : (f32x4){0.f, 0.f, 0.f, 0.f};
      } else {
        // (rows of other widths: four 4-B reads -- conflict-free for odd D -- then one 16-B
        // write per quad of the record; per-float writes at the record stride conflicted)
        const float* src = obs_s + t * a.D;
        for (int k = 0; k < a.D8; k += 4)
          *(f32x4*)(r + k) = (f32x4){k < a.D ? src[k] : 0.f, k + 1 < a.D ? src[k + 1] : 0.f,
                                     k + 2 < a.D ? src[k + 2] : 0.f, k + 3 < a.D ? src[k + 3] : 0.f};
      }
      float adv = a.adv[i];
      if (a.advantage_norm) adv = (adv - mean) / denom;  // ppo.py:243, fp32 as the reference
      if (a.adv_out) a.adv_out[i] = adv;
      *(f32x4*)(r + a.D8) = (f32x4){a.continuous ? 0.0f : __int_as_float(((const int32_t*)a.actions)[i]),
                                    a.logp[i], adv, a.ret[i]};
      if (a.continuous) {
        const int na = a.R - a.D8 - 4;  // a multiple of 4
        const float* sa = act_s + t * a.A;
        for (int k = 0; k < na; k += 4)
          *(f32x4*)(r + a.D8 + 4 + k) = (f32x4){k < a.A ? sa[k] : 0.f, k + 1 < a.A ? sa[k + 1] : 0.f,
                                                k + 2 < a.A ? sa[k + 2] : 0.f, k + 3 < a.A ? sa[k + 3] : 0.f};
      }
    }
    __syncthreads();
    // the tile's records are contiguous in memory: ns * R floats, R a multiple of 4
    f32x4* dst = (f32x4*)(a.rec + i0 * a.R);
    const f32x4* src = (const f32x4*)rec_s;
    for (int c = t; c < ns * a.R / 4; c += kPackTile) dst[c] = src[c];
    __syncthreads();
  }
}

inline int grid_for(int64_t n, int threads, int cap = 2048) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

}  // namespace

#ifdef DPPO_GAE_TRACE
extern "C" __attribute__((visibility("default"))) int dppo_debug_gae_trace(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gae_trace), sizeof(g_gae_trace)) == hipSuccess ? 0
                                                                                            : -2;
}
#endif

// gae_pipe_kernel<E, NT> for the DPPO_GAE_NT variant
template <int E, int NT>
int launch_pipe_nt(int grid, hipStream_t s, const float* r, const uint8_t* te, const uint8_t* tr,
                   const float* v, const float* nv, float* adv, float* ret, double* partials,
                   int T, int N, float gamma, float c, int wt, int stagger, int psleep) {
  const auto kern = gae_pipe_kernel<E, NT>;
  DPPO_LAUNCH(kern, dim3(grid), dim3(kPThreads), 0, s, r, te, tr, v, nv, adv, ret, partials, T,
              N, gamma, c, wt, stagger, psleep);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}
template <int E>
int launch_pipe(int nt, int grid, hipStream_t s, const float* r, const uint8_t* te,
                const uint8_t* tr, const float* v, const float* nv, float* adv, float* ret,
                double* partials, int T, int N, float gamma, float c, int wt, int stagger,
                int psleep) {
  switch (nt) {
    case 1: return launch_pipe_nt<E, 1>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 5: return launch_pipe_nt<E, 5>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 8: return launch_pipe_nt<E, 8>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 12: return launch_pipe_nt<E, 12>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 3: return launch_pipe_nt<E, 3>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 4: return launch_pipe_nt<E, 4>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    case 7: return launch_pipe_nt<E, 7>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
    default: return launch_pipe_nt<E, 0>(grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep);
  }
}

int launch_gae(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
               const float* nv, float* adv, float* ret, double* partials, int T, int N,
               float gamma, float gae_lambda, hipStream_t s, int* n_partials, int mode) {
  const int G = (N + kEnvTile - 1) / kEnvTile;
  *n_partials = G;
  if (T <= 0 || N <= 0) return DPPO_OK;
  // Python evaluates gamma * gae_lambda first, in double (ppo.py:214-216).
  const float c = (float)((double)gamma * (double)gae_lambda);
  const bool vec = (N % kEnvTile) == 0 && ((uintptr_t)r % 16 == 0) && ((uintptr_t)v % 16 == 0) &&
                   ((uintptr_t)nv % 16 == 0) && ((uintptr_t)adv % 16 == 0) &&
                   ((uintptr_t)ret % 16 == 0) && ((uintptr_t)te % 16 == 0) &&
                   ((uintptr_t)tr % 16 == 0);
  // DPPO_GAE_STAGED=1 selects the earlier stage-all / scan / store-all kernel (A/B timing only)
  static const bool staged = std::getenv("DPPO_GAE_STAGED") != nullptr;
  if (vec && !staged) {
    // persistent: at most one workgroup per CU, a multiple of 16 so XCD pairs stay aligned
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus <= 0)
        cus = 256;
    }
    // DPPO_GAE_E / DPPO_GAE_WGS_PER_CU: tile width and residency overrides (A/B timing only)
    static const int env_e = std::getenv("DPPO_GAE_E") ? std::atoi(std::getenv("DPPO_GAE_E")) : 0;
    static const int per_cu =
        std::getenv("DPPO_GAE_WGS_PER_CU") ? std::atoi(std::getenv("DPPO_GAE_WGS_PER_CU")) : 1;
    const bool e32 = env_e == 32 ? N % 32 == 0 : (env_e == 16 ? false : (N % 32 == 0 && N / 32 >= cus));
    // 64-env tiles (256-B rows) where they still give every CU a tile (N >= 16,384 on 256 CUs):
    // at N = 65,536 41.0 us per launch against 43.6 with 32-env tiles (exact mode, same box)
    const bool e64 = N % 64 == 0 && (env_e == 64 || (env_e == 0 && N / 64 >= cus));
    // DPPO_GAE_WT=0/1: plain or write-through (sc1) advantage / return stores (A/B timing)
    static const int wt = std::getenv("DPPO_GAE_WT") ? std::atoi(std::getenv("DPPO_GAE_WT")) : 0;
    // Cycles between the owners' first load bursts: 450-750 measured 8.0-8.25 us per launch at
    // N = 8192 against 9.1 without (1,200: 9.6, 1,800: 10.6).  DPPO_GAE_STAGGER overrides (A/B).
    static const int stagger =
        std::getenv("DPPO_GAE_STAGGER") ? std::atoi(std::getenv("DPPO_GAE_STAGGER")) : 640;
    // The scan wave's back-off between unsuccessful polls (s_sleep 1): 7.67-7.98 against
    // 7.90-8.19 us per launch at N = 8192 (rocprof, 3 A/B reps; s_sleep 2: 8.01-8.32).
    // DPPO_GAE_PSLEEP=0/1/2 overrides (A/B).
    static const int psleep =
        std::getenv("DPPO_GAE_PSLEEP") ? std::atoi(std::getenv("DPPO_GAE_PSLEEP")) : 1;
    // DPPO_GAE_NT: the owners' streaming variant (gae_pipe_kernel NT bits; 0, 1, 3, 4, 5, 7, 8 or
    // 12; A/B).
    // On cold rotating buffers (tools/gae_bench.py) non-temporal operand loads and advantage /
    // return stores (3) measured 7.25-7.59 against 7.73-7.84 us per launch at N = 8192; inside a
    // learn, where the eval kernel has just written values / next_values and the pack kernel reads
    // the advantages next, they cost: GAE 8.2-8.3 against 7.0-7.25 us, pack 23.7-24.8 against
    // 19.4 us at C3 (tools/gpu/r05_gae_nt_learn.sh).  Plain accesses stay the default.
    static const int nt = std::getenv("DPPO_GAE_NT") ? std::atoi(std::getenv("DPPO_GAE_NT")) : 0;
    const int tiles = e64 ? N / 64 : (e32 ? N / 32 : G);
    int grid = tiles < per_cu * cus ? tiles : per_cu * cus;
    if (!e32 && grid >= 16) grid -= grid % 16;
    *n_partials = grid;
    if (e64) {
      if (mode == DPPO_GAE_AFFINE)
        DPPO_LAUNCH(gae_aff_kernel<64>, dim3(grid), dim3(kPChunks * kWave), 0, s, r, te, tr, v,
                    nv, adv, ret, partials, T, N, gamma, c, stagger);
      else
        { const int rc_ = launch_pipe<64>(nt, grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep); if (rc_ != DPPO_OK) return rc_; }
    } else if (mode == DPPO_GAE_AFFINE) {
      if (e32)
        DPPO_LAUNCH(gae_aff_kernel<32>, dim3(grid), dim3(kPChunks * kWave), 0, s, r, te, tr, v,
                    nv, adv, ret, partials, T, N, gamma, c, stagger);
      else
        DPPO_LAUNCH(gae_aff_kernel<16>, dim3(grid), dim3(kPChunks * kWave), 0, s, r, te, tr, v,
                    nv, adv, ret, partials, T, N, gamma, c, stagger);
    } else if (e32)
      { const int rc_ = launch_pipe<32>(nt, grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep); if (rc_ != DPPO_OK) return rc_; }
    else
      { const int rc_ = launch_pipe<16>(nt, grid, s, r, te, tr, v, nv, adv, ret, partials, T, N, gamma, c, wt, stagger, psleep); if (rc_ != DPPO_OK) return rc_; }
  } else if (vec)
    DPPO_LAUNCH(gae_kernel<true>, dim3(G), dim3(kThreads), 0, s, r, te, tr, v, nv, adv, ret,
                       partials, T, N, gamma, c);
  else
    DPPO_LAUNCH(gae_kernel<false>, dim3(G), dim3(kThreads), 0, s, r, te, tr, v, nv, adv,
                       ret, partials, T, N, gamma, c);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

// ---- The streaming ceiling of the GAE launch (measurement only, dppo_gae_stream_probe): the
// same 22 B per element over the same [T][N] buffers -- read rewards, values, next_values (16 B
// per lane) and the two flag bytes, write advantages and returns -- with no recurrence, in the
// fastest pattern measured for one cold launch of these bytes (tools/probe/stream_probe2.hip, mode
// 7: non-temporal loads and stores, two elements per thread, each XCD's blocks on one contiguous
// eighth of the buffers; 6.4 against 7.6 us for plain accesses at N = 8192).  What one launch of
// these bytes reaches on this part (bench.py roofline_gae: ceiling_us, frac_of_ceiling).
__global__ __launch_bounds__(256) void gae_stream_probe_kernel(
    const float* __restrict__ r, const uint8_t* __restrict__ te, const uint8_t* __restrict__ tr,
    const float* __restrict__ v, const float* __restrict__ nv, float* __restrict__ adv,
    float* __restrict__ ret, int64_t n4) {
  const int64_t g = gridDim.x;
  const int64_t b = (g % 8 == 0) ? ((int64_t)blockIdx.x % 8) * (g / 8) + blockIdx.x / 8
                                 : (int64_t)blockIdx.x;
  const int64_t per = n4 / 2;
  for (int64_t i = b * 256 + threadIdx.x; i < per; i += g * 256) {
    f32x4 a[2], bb[2], c[2];
    uint32_t t[2], u[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t k = i + e * per;
      a[e] = __builtin_nontemporal_load((const f32x4*)r + k);
      bb[e] = __builtin_nontemporal_load((const f32x4*)v + k);
      c[e] = __builtin_nontemporal_load((const f32x4*)nv + k);
      t[e] = __builtin_nontemporal_load((const uint32_t*)te + k);
      u[e] = __builtin_nontemporal_load((const uint32_t*)tr + k);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t k = i + e * per;
      f32x4 o = c[e];
      o[0] += (float)((t[e] ^ u[e]) & 0xffu);
      __builtin_nontemporal_store(a[e] + bb[e], (f32x4*)adv + k);
      __builtin_nontemporal_store(o, (f32x4*)ret + k);
    }
  }
  // (n4 odd: the last element)
  if ((n4 & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t k = n4 - 1;
    f32x4 o = ((const f32x4*)nv)[k];
    o[0] += (float)((((const uint32_t*)te)[k] ^ ((const uint32_t*)tr)[k]) & 0xffu);
    ((f32x4*)adv)[k] = ((const f32x4*)r)[k] + ((const f32x4*)v)[k];
    ((f32x4*)ret)[k] = o;
  }
}

int launch_gae_stream_probe(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
                            const float* nv, float* adv, float* ret, int64_t n, hipStream_t s) {
  if (n <= 0) return DPPO_OK;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  const int64_t n4 = n / 4;
  int64_t grid = (n4 / 2 + 255) / 256;
  if (grid > 2 * cus) grid = 2 * cus;  // 512 on 256 CUs (stream_probe2: 256 and 512 level)
  if (grid >= 8) grid -= grid % 8;
  if (grid < 1) grid = 1;
  DPPO_LAUNCH(gae_stream_probe_kernel, dim3((unsigned)grid), dim3(256), 0, s, r, te, tr, v, nv,
              adv, ret, n4);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_stats_reduce(const double* partials, int n_partials, double* dsum, hipStream_t s) {
  DPPO_LAUNCH(stats_reduce_kernel, dim3(1), dim3(256), 0, s, partials, n_partials, dsum);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_stats_finalize(const double* dsum, double n_total, float* mean_std, hipStream_t s) {
  DPPO_LAUNCH(stats_finalize_kernel, dim3(1), dim3(64), 0, s, dsum, n_total, mean_std);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_adv_normalize(float* adv, const float* mean_std, int64_t n, hipStream_t s) {
  if (n <= 0) return DPPO_OK;
  DPPO_LAUNCH(adv_normalize_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, adv,
                     mean_std, n);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.B <= 0) return DPPO_OK;
  const size_t lds = (size_t)kPackTile * (a.D + (a.continuous ? a.A : 0) + a.R) * sizeof(float);
  // up to 100 KB at D = 32, A = 16
  static const bool attr = [] {
    raise_dyn_lds((const void*)pack_kernel);
    return true;
  }();
  (void)attr;
  DPPO_LAUNCH(pack_kernel, dim3(grid_for(a.B, kPackTile)), dim3(kPackTile), lds, s, a);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
