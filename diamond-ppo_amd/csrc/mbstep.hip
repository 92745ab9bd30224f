// Fused PPO minibatch step (gather -> forward -> loss -> analytic backward -> weight-gradient
// partials) on gfx950 fp32 MFMA: a two-team, software-pipelined workgroup.
//
// Reference: loss and backward of one minibatch, diamond/ppo.py:261-283 (continuous:
// continuous_ppo.py:273-295), default networks ppo.py:53-71 / continuous_ppo.py:63-81.
//
// ---- Decomposition ----------------------------------------------------------------------------
// A workgroup = 8 waves (512 threads, one workgroup per CU, two waves per SIMD) in two teams of
// four.  The minibatch is cut into steps of S = 32 samples.  In interval set `it`:
//   * team 0 (the FORWARD team) gathers step it, runs the hidden layers, the heads and the
//     per-sample loss, and back-propagates through the heads (VALU-heavy: tanh, softmax /
//     Gaussian log-prob, clipped surrogate);
//   * team 1 (the BACKWARD team) back-propagates step it-1 through the hidden layers and
//     accumulates the hidden weight gradients (MFMA-heavy).
// The two waves sharing a SIMD therefore overlap one team's VALU/LDS phases with the other
// team's MFMA chains.  Each team holds only its own weight slices in registers (forward: row
// slices of W1, W2, Wa, Wc; backward: column slices of W2, Wa, Wc) and team 1 alone holds the
// hidden weight-gradient accumulators, which keeps both under the 256-VGPR budget of two waves
// per SIMD.  Images handed from team 0 to team 1 (X0, H1, H2, dZ[a|c]) are double-buffered by
// step parity; every interval set has five workgroup barriers for both teams.
//
// Inside a team the hidden layers are split by OUTPUT feature: wave q owns features
// [16q, 16q+16) of every layer, for every sample of the step:
//   * forward  Y[16q.., s] = W[16q.., :] X[:, s]      A = its 16-row slice of W (registers),
//   * backward dX[16q.., s] = W[:, 16q..]^T dZ[:, s]  A = its 16-column slice of W (registers),
//   * dW[16q.., :] += dZ[16q.., s] X[:, s]^T          accumulator: 16 rows x 64 = 16 registers,
// with v_mfma_f32_16x16x4_f32 (exact fp32).  The feature columns of every activation image are
// permuted inside each 16-column block, col(k) = 16(k>>4) + 4(k&3) + ((k>>2)&3), so that the 4
// consecutive k-steps a lane feeds the MFMA B operand are 16 contiguous bytes (one ds_read_b128
// per 4 MFMAs).  Heads (logits / Gaussian mean, value) and the per-sample loss run on VALU, 8
// lanes per sample.  Every accumulator is written once per workgroup into its slab (optim.hip
// sums the slabs in a fixed order): bit-reproducible, no float atomics.
#include "common.h"

namespace dppo {
namespace {

constexpr int H = 64;
constexpr int kTeamWaves = 4;
constexpr int kTeams = 2;
constexpr int kThreads = kTeams * kTeamWaves * kWave;  // 512: two waves per SIMD
constexpr int S = 32;                                   // samples per step
constexpr int NSB = S / 16;                             // 16-sample MFMA tiles per step
constexpr int NPASS = S / (kTeamWaves * 8);             // gather/head passes (8 lanes/sample)
constexpr int SPW = S / kTeamWaves;                     // samples per wave in the head phases
static_assert(NPASS == 1, "one gather/head pass per step");
static_assert(S == 32, "wgrad16 maps its 8 k-steps x 4 lane groups onto 32 samples");
constexpr int SA = 68;                                  // stride of 64-col images
constexpr int SAC = 132;                                // stride of the [ha | hc] images
constexpr int SD = 68;                                  // stride of the per-sample head image
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
constexpr float kLn2 = 0.69314718055994530942f;
constexpr float kHalfLog2PiPlusHalf = 1.41893853320467274178f;

// Timing-only ablation switches (tools/ablate.py); a shipped build defines none of them.
#ifdef DPPO_ABL_NOBARRIER
#define STEP_BARRIER() __builtin_amdgcn_wave_barrier()
#define HEAD_STAMP(k) \
  do {                \
  } while (0)
#elif defined(DPPO_PHASE_TRACE)
// Timing-only build: workgroup 0 records, per wave and per barrier, the cycle counter when the
// wave arrives (its phase work issued and drained) and when the barrier releases it.
constexpr int kTraceBars = 128;
__device__ long long g_phase_trace[kTraceBars][kThreads / 64][2];
// per workgroup: s_memtime at entry, loop entry, loop exit, epilogue drained; s_memrealtime at
// entry and at the end (cross-CU skew)
__device__ long long g_phase_edges[256][6];
#define EDGE_STAMP(i)                                                                 \
  do {                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 256)                                         \
      g_phase_edges[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                    \
  } while (0)
#define EDGE_REAL(i)                                                                  \
  do {                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 256)                                         \
      g_phase_edges[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
__device__ long long g_heads_trace[kTraceBars][4];
#define HEAD_STAMP(k)                                                                   \
  do {                                                                                  \
    if (blockIdx.x == 0 && threadIdx.x == 0 && tr_k_ < kTraceBars)                     \
      g_heads_trace[tr_k_][k] = __builtin_amdgcn_s_memtime();                          \
  } while (0)
#define STEP_BARRIER()                                                        \
  do {                                                                        \
    __builtin_amdgcn_s_waitcnt(0xc07f); /* lgkmcnt(0) only, as __syncthreads */ \
    const long long t0_ = clock64();                                          \
    __syncthreads();                                                          \
    const long long t1_ = clock64();                                          \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && tr_k_ < kTraceBars) {   \
      g_phase_trace[tr_k_][threadIdx.x >> 6][0] = t0_;                        \
      g_phase_trace[tr_k_][threadIdx.x >> 6][1] = t1_;                        \
    }                                                                         \
    ++tr_k_;                                                                  \
  } while (0)
#else
#define STEP_BARRIER() __syncthreads()
#define HEAD_STAMP(k) \
  do {                \
  } while (0)
#endif
#ifndef EDGE_STAMP
#define EDGE_STAMP(i) \
  do {                \
  } while (0)
#define EDGE_REAL(i) \
  do {               \
  } while (0)
#endif

__host__ __device__ constexpr int perm(int k) { return (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3); }

struct Lds2 {  // offsets (floats)
  int Wo;                  // [16][64] head weights, permuted columns
  int Wv;                  // [64] permuted
  int b1, b2, ba, bc;      // [64] natural order
  int bo, ls, bv;          // [16] [16] [4]
  int gc;                  // [4][16] Gaussian per-action constants (continuous), see prologue
  int gent;                // [4] {sum over actions of the Gaussian entropy terms}
  int PART;                // [4][S][16] per-wave partial head outputs (MFMA heads, AMAX == 8)
  int X0[2], H1[2], H2[2], DZAC[2];  // team 0 -> team 1 hand-off, double-buffered by step parity
  int HAC, DOUT;           // team 0 only: [ha | hc] activations, per-sample head deltas
  int DZ2, DZ1;            // team 1 only
  int SX0;                 // X0 stride
  int total;
};

struct MArgs {
  Lds2 L;
  ParamOffsets po;
  const float* params;
  const float* rec;
  const int32_t* idx;
  const int32_t* seg;  // global-minibatch DP: {start, end} of this minibatch in idx (device)
  int m;
  float inv_m, clip_eps, vf, ent;
  float* slabs;
  int64_t slab_stride, p_total;
  int D, D8, D16, A, R;
  int fuse;      // single device: the slab reduction, clip and Adam run in this launch's tail
  int nblk;      // 64-parameter blocks of the tail (slab_reduce_blocks)
  FusedAdam fa;
};

constexpr int kTailParams = 64;  // parameters per tail block (= optim.hip's kRedParams)

// Tail of a single-device launch (replaces reduce_adam_kernel and its launch): every workgroup's
// slab is published (sc1 stores, drained); after a grid fan-in workgroup b reduces parameter
// blocks b, b + G, ... over all G slabs (sc1 loads, wave w takes slabs w, w + 8, ...; the wave
// partials are combined in a fixed order), publishes them and each block's sum of squares; after
// a second fan-in every workgroup sums the block squares in the same order (global norm,
// clip_grad.py:165-169) and applies Adam (torch _single_tensor_adam op order) to its blocks.
__device__ void fused_reduce_adam(const MArgs& a, float* lds) {
#pragma clang fp contract(off)
  const FusedAdam& f = a.fa;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kThreads / 64;
  const int G = gridDim.x;
  const int64_t n = a.p_total + 8;
  int* released = (int*)(lds + NW * 64);  // thread 0's fan-in outcome, for the whole block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores are complete
  __syncthreads();
  if (tid == 0) *released = grid_fanin(f.arrivals, f.epoch, f.timeout_ticks, f.err) ? 1 : 0;
  __syncthreads();
  // a timed-out fan-in (grid not co-resident) leaves the parameters untouched; the handle's
  // sticky error word reports it at the next C-ABI call
  if (!*released) return;
  for (int blk = blockIdx.x; blk < a.nblk; blk += G) {
    const int64_t p = (int64_t)blk * kTailParams + lane;
    float sacc = 0.0f;
    if (p < n) {
      const float* src = a.slabs + p;
      int g = wave;
      for (; g + 15 * NW < G; g += 16 * NW) {
        float x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          x[k] = __hip_atomic_load(src + (int64_t)(g + NW * k) * a.slab_stride, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc += x[k];
      }
      for (; g < G; g += NW)
        sacc += __hip_atomic_load(src + (int64_t)g * a.slab_stride, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    lds[wave * 64 + lane] = sacc;
    __syncthreads();
    if (wave == 0) {
      float t = 0.0f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += lds[w * 64 + lane];
      // d(-beta * mean H)/d log_std = -beta per action dim (continuous_ppo.py:286-291)
      if (f.add_entropy_const && p >= f.ls_off && p < f.ls_off + f.ls_n) t -= a.ent;
      if (p < n) __hip_atomic_store(f.grad + p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      double q = (p < a.p_total) ? (double)t * (double)t : 0.0;
      for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
      if (lane == 0)
        __hip_atomic_store(f.sq_part + blk, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();  // lds reused by the next block
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    *released = grid_fanin(f.arrivals + kArrivalWords, f.epoch, f.timeout_ticks, f.err) ? 1 : 0;
  __syncthreads();
  if (wave != 0 || !*released) return;
  double sq = 0.0;
  for (int k = lane; k < a.nblk; k += 64)
    sq += __hip_atomic_load(f.sq_part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
  float norm;
  const float coef = clip_coef(sq, f.max_norm, &norm);
  for (int blk = blockIdx.x; blk < a.nblk; blk += G) {
    const int64_t p = (int64_t)blk * kTailParams + lane;
    if (p < a.p_total) {
      float pk = f.params[p], mk = f.m[p], vk = f.v[p];
      const float gk = __hip_atomic_load(f.grad + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      adam_regs(pk, gk, mk, vk, coef, 1.0f - f.beta1, 1.0f - f.beta2, f.beta2, f.bc2_sqrt, f.eps,
                f.neg_step_size);
      f.params[p] = pk;
      f.m[p] = mk;
      f.v[p] = vk;
    }
  }
  if (blockIdx.x == 0 && lane == 0 && f.trace) {
    const float* ls = f.grad + a.p_total;
    write_trace(f.trace, __hip_atomic_load(ls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(ls + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(ls + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), norm,
                a.inv_m, a.vf, a.ent);
  }
}

inline int a4(int x) { return (x + 3) & ~3; }

__device__ __forceinline__ void zero_image(float* img, int n4, int tid) {
  for (int c = tid; c < n4; c += kThreads) ((f32x4*)img)[c] = (f32x4){0.f, 0.f, 0.f, 0.f};
}

Lds2 make_lds2(int D16) {
  Lds2 L{};
  int o = 0;
  auto take = [&](int n) {
    const int r = o;
    o += a4(n);
    return r;
  };
  L.Wo = take(16 * H);
  L.Wv = take(H);
  L.b1 = take(H);
  L.b2 = take(H);
  L.ba = take(H);
  L.bc = take(H);
  L.bo = take(16);
  L.ls = take(16);
  L.bv = take(4);
  L.gc = take(4 * 16);
  L.gent = take(4);
  L.SX0 = D16 + 4;
  for (int b = 0; b < 2; ++b) {
    L.X0[b] = take(S * L.SX0);
    L.H1[b] = take(S * SA);
    L.H2[b] = take(S * SA);
    L.DZAC[b] = take(S * SAC);
  }
  L.HAC = take(S * SAC);
  L.PART = take(kTeamWaves * S * 16);
  L.DOUT = take(S * SD);
  L.DZ2 = take(S * SA);
  L.DZ1 = take(S * SA);
  L.total = o;
  return L;
}

// Per-iteration opaque LDS base: keeps loop-invariant LDS reads (head weights, biases) next to
// their uses instead of hoisted into registers for the whole kernel.
__device__ __forceinline__ float* opaque_base(float* p) {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return p + z;
}

// Slab stores are write-through (sc1): the ~13 MB of per-workgroup gradient partials leave the
// XCD L2s while the kernel runs instead of as dirty lines at the kernel boundary, and the reduce
// kernel (other XCDs) reads them from memory either way (MI355X_MICROARCH.md: boundary,
// publish-large).
__device__ __forceinline__ void slab_put4(float* p, f32x4 v) {
#ifdef DPPO_ABL_PLAINSLAB
  *(f32x4*)p = v;
#else
  // s_nop: a VALU write to the data VGPRs of a store wider than 8 bytes needs a wait state
  // after it, which the compiler cannot insert behind an asm statement (seen: back-to-back slab
  // stores whose next operands overwrote this one's data before it was read)
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#endif
}

// Register-slice staging of the hidden weights (prologue): W2, Wa, Wc land in LDS through
// coalesced 16-B loads (every workgroup reads the same 48 KB: one request per 1 KB wave-load
// instead of sixteen 16-B pieces per 4-B lane load), rows padded to kStageRow floats so that both
// the row slices of the forward team (lane (l15, h4) reads row 16q + l15, columns 4t + h4) and the
// column slices of the backward team (row 4t + h4, column 16q + l15) are near conflict-free b32
// reads (kStageRow = 18 mod 32).
constexpr int kStageRow = 82;
constexpr int kStageFloats = 3 * H * kStageRow;
// The epilogue assembles the workgroup's gradient slab in LDS (after the head-partial scratch of
// the forward team) and writes it out as 16-B write-through stores.
constexpr int kEpiHead = kTeamWaves * (16 + 3) * 64;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Sum over each aligned group of 8 lanes, the result in all 8 lanes, with DPP lane moves (VALU
// operand modifiers) instead of ds_bpermute round trips through the LDS unit.  The adds pair
// lanes exactly as x += shfl_xor(x, 1); x += shfl_xor(x, 2); x += shfl_xor(x, 4) would.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum8(float x) {
  x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]: lane ^ 1
  x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]: lane ^ 2
  x += dpp_mov<0x141>(x);  // row_half_mirror: lane 7 - i of the 8-lane group (the other quad)
  return x;
}

// 8-term dot product as a balanced tree (3 dependent adds instead of 8): the head phase is a
// latency chain, not a throughput one
__device__ __forceinline__ float dot8(f32x4 w0, f32x4 w1, f32x4 x0, f32x4 x1) {
  const float a = w0[0] * x0[0] + w0[1] * x0[1], b = w0[2] * x0[2] + w0[3] * x0[3];
  const float c = w1[0] * x1[0] + w1[1] * x1[1], d = w1[2] * x1[2] + w1[3] * x1[3];
  return (a + b) + (c + d);
}

__device__ __forceinline__ float tanh_f(float x) {
  // tanh via one exp and one hardware reciprocal, branch-free: t = e^{-2|x|},
  // tanh = sign(x) (1 - t) / (1 + t).  Absolute error <= ~1.5e-7 over the whole range (1 - t
  // cancels near 0, which costs relative but not absolute accuracy; activations are O(1)).
#ifdef DPPO_ABL_NOTANH
  return x * 0.5f;
#endif
  const float t = __expf(-2.0f * fabsf(x));
  return copysignf((1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t), x);
}

// One 16-row output slice for the NSB sample tiles: acc[sb] += W(regs, k = 4t + h4) x X(LDS
// image).  Software-pipelined: the B operands of k-block q+1 are requested before the MFMAs of
// block q issue, so the LDS latency hides under 4 x NSB MFMAs (16x16x4 f32: 32-cycle issue).
template <int NT>
__device__ __forceinline__ void mm_rows(f32x4 (&acc)[NSB], const float (&w)[NT], const float* X,
                                        int stride, int l15, int h4) {
#ifdef DPPO_ABL_NOMM
  return;
#endif
  constexpr int NQ = NT / 4;
  f32x4 b[2][NSB];
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb)
    b[0][sb] = *(const f32x4*)(X + (16 * sb + l15) * stride + 4 * h4);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q + 1 < NQ) {
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
        b[(q + 1) & 1][sb] = *(const f32x4*)(X + (16 * sb + l15) * stride + 16 * (q + 1) + 4 * h4);
    }
    __builtin_amdgcn_sched_barrier(0);
    // consecutive MFMAs hit different accumulators (dependent latency > issue interval)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) acc[sb] = mfma16(w[4 * q + j], b[q & 1][sb][j], acc[sb]);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// mm_rows for a first layer of K = 4 * NT <= 16 inputs (one 16-column block): NT MFMAs per tile.
template <int NT>
__device__ __forceinline__ void mm_rows_lo(f32x4 (&acc)[NSB], const float (&w)[8], const float* X,
                                           int stride, int l15, int h4) {
  f32x4 b[NSB];
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) b[sb] = *(const f32x4*)(X + (16 * sb + l15) * stride + 4 * h4);
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) acc[sb] = mfma16(w[j], b[sb][j], acc[sb]);
}

// Write a wave's output rows (16q + 4h4 + r, sample 16sb + l15) into an image (permuted cols).
__device__ __forceinline__ void put_rows(float* X, int stride, int col0, const f32x4 (&v)[NSB],
                                         int l15, int h4) {
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) {
    float* p = X + (16 * sb + l15) * stride + col0 + h4;
#pragma unroll
    for (int r = 0; r < 4; ++r) p[4 * r] = v[sb][r];
  }
}

// Read back a wave's own rows from an image (the positions put_rows wrote).
__device__ __forceinline__ void get_rows(f32x4 (&v)[NSB], const float* X, int stride, int col0,
                                         int l15, int h4) {
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) {
    const float* p = X + (16 * sb + l15) * stride + col0 + h4;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[sb][r] = p[4 * r];
  }
}

__device__ __forceinline__ void init_bias(f32x4 (&acc)[NSB], const float* b, int row0, int h4) {
  const f32x4 bb = *(const f32x4*)(b + row0 + 4 * h4);
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) acc[sb] = bb;
}

__device__ __forceinline__ void zero(f32x4 (&acc)[NSB]) {
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb) acc[sb] = (f32x4){0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void tanh_rows(f32x4 (&v)[NSB]) {
#pragma unroll
  for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
#ifdef DPPO_ABL_NOTANH
      v[sb][r] *= 0.5f;
      v[sb][r + 1] *= 0.5f;
#else
      const f32x2 y = tanh2((f32x2){v[sb][r], v[sb][r + 1]});
      v[sb][r] = y[0];
      v[sb][r + 1] = y[1];
#endif
    }
}

// dW rows (16q..) += sum over the S staged samples: A = dZ image (cols perm(o)), B = X image
// (k = sample).  Operands are prefetched two k-steps ahead of their MFMAs.
template <int NIB>
__device__ __forceinline__ void wgrad16(f32x4* acc, const float* DZ, int dz_stride,
                                        int dz_col0, const float* X, int x_stride, int x_col0,
                                        int row0, int l15, int h4) {
#ifdef DPPO_ABL_NOWGRAD
  return;
#endif
  constexpr int NT = S / 4;
  constexpr int PD = 2;  // prefetch distance
  const int ca = dz_col0 + perm(row0 + l15);
  float av[PD + 1], bv[PD + 1][NIB];
  // k-step t of lane group h4 takes sample (t & 3) + 4 h4 + 16 (t >> 2): any bijection onto the
  // step's samples sums the same terms, and this one puts lane groups h4 and h4 + 1 four rows
  // apart, i.e. 16 banks apart at every image stride used (== 4 mod 32): conflict-free b32 reads
  auto load = [&](int t, int slot) {
    const int s = (t & 3) + 4 * h4 + 16 * (t >> 2);
    av[slot] = DZ[s * dz_stride + ca];
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib) bv[slot][ib] = X[s * x_stride + x_col0 + perm(16 * ib + l15)];
  };
#pragma unroll
  for (int t = 0; t < PD; ++t) load(t, t);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t + PD < NT) load(t + PD, (t + PD) % (PD + 1));
    __builtin_amdgcn_sched_barrier(0);
    const int sl = t % (PD + 1);
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib) acc[ib] = mfma16(av[sl], bv[sl][ib], acc[ib]);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 1) void mb_kernel(MArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int team = wave / kTeamWaves;
  const int q = wave % kTeamWaves;  // feature quarter owned by this wave within its team
  const int l15 = lane & 15, h4 = lane >> 4;
  const Lds2& L = a.L;
  const float* P = a.params;
  const ParamOffsets& po = a.po;
  const int row0 = 16 * q;  // this wave's feature rows
  const int SX0 = L.SX0;
  const int nk1 = a.D16 / 4;  // layer-1 k-steps (4 or 8)
  // this rank's share of a global minibatch is known only on the device (shard_select, shuffle.hip)
  int mm = a.m;
  const int32_t* idxp = a.idx;
  if (a.seg) {
    const int s0 = a.seg[0];
    mm = a.seg[1] - s0;
    idxp += s0;
  }
  const int nsteps = (mm + S - 1) / S;
  const int nit = (nsteps + (int)gridDim.x - 1) / (int)gridDim.x;  // steps per workgroup
  float* slab = a.slabs + (int64_t)blockIdx.x * a.slab_stride;
  EDGE_STAMP(0);
  EDGE_REAL(4);
  // forward team: the first step's sample index before anything else (its record gather waits on
  // it); lane group (lane >> 3) of wave q takes sample 8 q + (lane >> 3) of a step
  const int hs = SPW * q + (lane >> 3);
  int nidx0 = 0;
  if (team == 0 && nit > 0 && (int)blockIdx.x * S + hs < mm) nidx0 = idxp[(int)blockIdx.x * S + hs];

  // ---------------- prologue: LDS head weights / biases
  for (int k = tid; k < 16 * H; k += kThreads) {
    const int r = k >> 6, f = k & 63;
    lds_[L.Wo + r * H + perm(f)] = r < a.A ? P[po.Wo + r * H + f] : 0.0f;
  }
  for (int k = tid; k < H; k += kThreads) {
    lds_[L.Wv + perm(k)] = P[po.Wv + k];
    lds_[L.b1 + k] = P[po.b1 + k];
    lds_[L.b2 + k] = P[po.b2 + k];
    lds_[L.ba + k] = P[po.ba + k];
    lds_[L.bc + k] = P[po.bc + k];
  }
  for (int k = tid; k < 16; k += kThreads) {
    lds_[L.bo + k] = k < a.A ? P[po.bo + k] : 0.0f;
    lds_[L.ls + k] = (po.ls >= 0 && k < a.A) ? P[po.ls + k] : 0.0f;
  }
  if (tid < 4) lds_[L.bv + tid] = tid == 0 ? P[po.bv] : 0.0f;
  if (CONT && tid < 16) {
    // Normal(mean, exp(log_std)) constants of action k, the same for every sample: computed once
    // per minibatch instead of an exp, a log and IEEE divisions per sample and action
    // (continuous_ppo.py:41-47; torch Normal.log_prob / entropy)
    const bool on = po.ls >= 0 && tid < a.A;
    const float sg = on ? __expf(P[po.ls + tid]) : 1.0f;
    const float lsc = on ? __logf(sg) : 0.0f;
    lds_[L.gc + tid] = on ? 1.0f / (2.0f * (sg * sg)) : 0.0f;  // 1 / (2 var), 0 past A
    lds_[L.gc + 16 + tid] = 1.0f / (sg * sg);       // 1 / var
    lds_[L.gc + 32 + tid] = 1.0f / sg;              // 1 / sigma
    lds_[L.gc + 48 + tid] = lsc;                    // log sigma
    if (tid == 0) {
      float e = 0.0f, c = 0.0f;
      for (int k = 0; k < a.A && k < 16; ++k) {
        const float l = __logf(__expf(P[po.ls + k]));
        e += kHalfLog2PiPlusHalf + l;  // entropy (continuous_ppo.py:45-47)
        c += l + kLogSqrt2Pi;          // log-prob constant part
      }
      lds_[L.gent] = e;
      lds_[L.gent + 1] = c;
    }
  }

  {
    // W2 | Wa | Wc -> padded LDS image (the step-image area, unused until the main loop)
    float* stg = lds_ + L.H1[0];
    for (int k = tid; k < 3 * H * H / 4; k += kThreads) {
      const int m = k >> 10, e = k & 1023, row = e >> 4, c4 = e & 15;
      const int off = m == 0 ? po.W2 : (m == 1 ? po.Wa : po.Wc);
      const f32x4 v = *(const f32x4*)(P + off + row * H + 4 * c4);
      float* d = stg + m * H * kStageRow + row * kStageRow + 4 * c4;
      *(f32x2*)d = (f32x2){v[0], v[1]};
      *(f32x2*)(d + 2) = (f32x2){v[2], v[3]};
    }
  }
  __syncthreads();
  const float* stg = lds_ + L.H1[0];
  float* img = lds_ + kEpiHead;                       // epilogue: this workgroup's slab image
  const int nimg4 = (int)((a.p_total + 8 + 3) / 4);   // parameters + loss slots, in f32x4

  if (team == 0) {
    // =========================== forward team ===========================
    float w1f[8], w2f[16], waf[16], wcf[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int k = 4 * t + h4;
      w1f[t] = k < a.D ? P[po.W1 + (row0 + l15) * a.D + k] : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int k = 4 * t + h4;
      const int o = (row0 + l15) * kStageRow + k;
      w2f[t] = stg[o];
      waf[t] = stg[H * kStageRow + o];
      wcf[t] = stg[2 * H * kStageRow + o];
    }
    f32x4 gba = (f32x4){0.f, 0.f, 0.f, 0.f}, gbc = gba;  // hidden-bias partials (ba, bc rows)
    float gWo[AMAX];
#pragma unroll
    for (int k = 0; k < AMAX; ++k) gWo[k] = 0.f;
    float gWv = 0.f, gbh = 0.f, s_pi = 0.f, s_v = 0.f, s_ent = 0.f;
    const int hj = lane & 7;             // 8 lanes per sample

    // Sample-record prefetch: after the heads of step it the records of step it+1 (observation
    // chunk, {action, old log-prob, advantage, return}, continuous actions) and the indices of step
    // it+2 are requested; the records are gathered at random (latency, not bandwidth).
    constexpr int NA4 = CONT ? (AMAX + 3) / 4 : 1;
    int nidx = 0;
    f32x4 pobs, psc, pact[NA4];   // records of the next step (in flight)
    f32x4 csc, cact[NA4];          // {action bits, old log-prob, adv, return} of the current step
    auto load_idx = [&](int it) {
      const int step = it * (int)gridDim.x + (int)blockIdx.x;
      const int si = step * S + hs;
      nidx = (it < nit && si < mm) ? idxp[si] : 0;
    };
    auto load_rec = [&](int it) {
      const int step = it * (int)gridDim.x + (int)blockIdx.x;
      const int si = step * S + hs;
      const bool valid = it < nit && si < mm;
      const float* rec = a.rec + (int64_t)nidx * a.R;
      pobs = (valid && hj < nk1 && 4 * hj < a.D8) ? *(const f32x4*)(rec + 4 * hj)
                                                 : (f32x4){0.f, 0.f, 0.f, 0.f};
      psc = *(const f32x4*)(rec + a.D8);
#pragma unroll
      for (int c = 0; c < NA4; ++c)
        pact[c] = (CONT && 4 * c < a.A) ? *(const f32x4*)(rec + a.D8 + 4 + 4 * c)
                                        : (f32x4){0.f, 0.f, 0.f, 0.f};
    };
    // gather: observation chunk of the prefetched record -> X0 of step `it` (permuted cols)
    auto gather = [&](int it) {
      if (it < nit && hj < nk1) {
        float* X0 = lds_ + L.X0[it & 1];
        const int kb = 4 * hj;
#pragma unroll
        for (int j = 0; j < 4; ++j) X0[hs * SX0 + perm(kb + j)] = pobs[j];
      }
    };
    nidx = nidx0;  // load_idx(0), issued at kernel entry
    load_rec(0);
    csc = psc;
#pragma unroll
    for (int c = 0; c < NA4; ++c) cact[c] = pact[c];
    gather(0);
    load_idx(1);
    __syncthreads();  // LDS head weights / biases and X0 of step 0 visible
    EDGE_STAMP(1);
    // Up to 4 actions the head weights this lane touches are loop-invariant registers: in the
    // head phase lane hj covers permuted columns [4hj, 4hj+4) and [32+4hj, 32+4hj+4) of a
    // sample; in the head back-propagation it covers the permuted columns of its own rows.
    // (Rows k >= A of the LDS head image are zero.)
    constexpr bool WREG = AMAX <= 4;
    constexpr int AR = WREG ? AMAX : 1;
    float woh[AR][8], wvh[8], wod[AR][4], wvd[4];
    if (WREG) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int k = 0; k < AR; ++k) {
          woh[k][j] = lds_[L.Wo + k * H + 4 * hj + j];
          woh[k][4 + j] = lds_[L.Wo + k * H + 32 + 4 * hj + j];
          wod[k][j] = lds_[L.Wo + k * H + row0 + 4 * j + h4];
        }
        wvh[j] = lds_[L.Wv + 4 * hj + j];
        wvh[4 + j] = lds_[L.Wv + 32 + 4 * hj + j];
        wvd[j] = lds_[L.Wv + row0 + 4 * j + h4];
      }
    }
    // MFMA heads (AMAX == 8, up to 8 actions): the head outputs are [16 rows = A logits / means,
    // row 8 = value] x samples.  Each wave multiplies the 16 head-input features it owns (its rows
    // of ha and hc, already in registers after interval 3) -- 8 v_mfma_f32_16x16x4_f32 per sample
    // tile, A = its Wo / Wv columns, B = its activation registers -- and leaves the partial in
    // LDS; the heads phase sums the four partials instead of 8-lane dot products + DPP trees.
    // The head back-propagation dZa = Wo^T dout is two MFMA k-steps on the same layout.
    constexpr bool MH = AMAX == 8;
    float woA[MH ? 4 : 1], wvA[MH ? 4 : 1], woT[MH ? 2 : 1];
    if (MH) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = row0 + 4 * h4 + r;
        woA[r] = l15 < a.A ? P[po.Wo + l15 * H + f] : 0.0f;
        wvA[r] = l15 == AMAX ? P[po.Wv + f] : 0.0f;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int k = 4 * t + h4;
        woT[t] = k < a.A ? P[po.Wo + k * H + row0 + l15] : 0.0f;
      }
    }
#ifdef DPPO_PHASE_TRACE
    int tr_k_ = 0;
#endif

    for (int it = 0; it <= nit; ++it) {
      const bool act = it < nit;
      const int b = it & 1;
      const int step = it * (int)gridDim.x + (int)blockIdx.x;
      float* lds = opaque_base(lds_);
      float* X0 = lds + L.X0[b];
      float* H1 = lds + L.H1[b];
      float* H2 = lds + L.H2[b];
      float* HAC = lds + L.HAC;
      float* DOUT = lds + L.DOUT;
      float* DZAC = lds + L.DZAC[b];
      // ---- (1) layer 1
      if (act) {
        f32x4 h1r[NSB];
        init_bias(h1r, lds + L.b1, row0, h4);
        // k-steps t cover inputs 4t .. 4t+3: only ceil(D/4) of them are non-zero
        if (a.D > 16) mm_rows<8>(h1r, w1f, X0, SX0, l15, h4);
        else if (a.D > 12) mm_rows_lo<4>(h1r, w1f, X0, SX0, l15, h4);
        else if (a.D > 8) mm_rows_lo<3>(h1r, w1f, X0, SX0, l15, h4);
        else if (a.D > 4) mm_rows_lo<2>(h1r, w1f, X0, SX0, l15, h4);
        else mm_rows_lo<1>(h1r, w1f, X0, SX0, l15, h4);
        tanh_rows(h1r);
        put_rows(H1, SA, row0, h1r, l15, h4);
      }
      STEP_BARRIER();
      // ---- (2) layer 2
      if (act) {
        f32x4 h2r[NSB];
        init_bias(h2r, lds + L.b2, row0, h4);
        mm_rows<16>(h2r, w2f, H1, SA, l15, h4);
        tanh_rows(h2r);
        put_rows(H2, SA, row0, h2r, l15, h4);
      }
      STEP_BARRIER();
      // ---- (3) actor / critic hidden layers
      if (act) {
        f32x4 har[NSB], hcr[NSB];
        init_bias(har, lds + L.ba, row0, h4);
        init_bias(hcr, lds + L.bc, row0, h4);
        mm_rows<16>(har, waf, H2, SA, l15, h4);
        mm_rows<16>(hcr, wcf, H2, SA, l15, h4);
        tanh_rows(har);
        tanh_rows(hcr);
        put_rows(HAC, SAC, row0, har, l15, h4);
        put_rows(HAC, SAC, 64 + row0, hcr, l15, h4);
        if (MH) {
          float* part = lds + L.PART + q * S * 16;
#pragma unroll
          for (int sb = 0; sb < NSB; ++sb) {
            f32x4 o = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 4; ++r) o = mfma16(woA[r], har[sb][r], o);
#pragma unroll
            for (int r = 0; r < 4; ++r) o = mfma16(wvA[r], hcr[sb][r], o);
            // lane (sample 16 sb + l15, h4) holds head rows 4 h4 .. 4 h4 + 3
            *(f32x4*)(part + (16 * sb + l15) * 16 + 4 * h4) = o;
          }
        }
      }
      STEP_BARRIER();
      // ---- (4) heads + loss (VALU, 8 lanes per sample)
#ifdef DPPO_ABL_NOHEADS
      if (step < 0)
#endif
      if (act) {
        const int si = step * S + hs;
        const bool valid = si < mm;
        const f32x4 sc = csc;  // {action bits, old logp, adv, return}
        const float* hrow = HAC + hs * SAC;
        const f32x4 ha0 = *(const f32x4*)(hrow + 4 * hj), ha1 = *(const f32x4*)(hrow + 32 + 4 * hj);
        const f32x4 hc0 = *(const f32x4*)(hrow + 64 + 4 * hj);
        const f32x4 hc1 = *(const f32x4*)(hrow + 96 + 4 * hj);
        // all AMAX rows, branch-free (head-image rows and biases k >= A are zero, so out[k] = 0):
        // the AMAX independent dot / DPP chains interleave instead of running one by one
        float out[AMAX];
        float vmh = 0.f;
        if (MH) {
          f32x4 s0 = (f32x4){0.f, 0.f, 0.f, 0.f}, s1 = s0;
          float sv = 0.f;
#pragma unroll
          for (int w = 0; w < kTeamWaves; ++w) {
            const float* pr = lds + L.PART + (w * S + hs) * 16;
            s0 += *(const f32x4*)pr;
            s1 += *(const f32x4*)(pr + 4);
            sv += pr[AMAX];
          }
#pragma unroll
          for (int k = 0; k < AMAX; ++k) out[k] = (k < 4 ? s0[k & 3] : s1[k & 3]) + lds[L.bo + k];
          vmh = sv;
        } else
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
          f32x4 w0, w1;
          if (WREG) {
            w0 = (f32x4){woh[k][0], woh[k][1], woh[k][2], woh[k][3]};
            w1 = (f32x4){woh[k][4], woh[k][5], woh[k][6], woh[k][7]};
          } else {
            w0 = *(const f32x4*)(lds + L.Wo + k * H + 4 * hj);
            w1 = *(const f32x4*)(lds + L.Wo + k * H + 32 + 4 * hj);
          }
          out[k] = sum8(dot8(w0, w1, ha0, ha1)) + lds[L.bo + k];
        }
        float vp = vmh;
        if (!MH) {
          f32x4 w0, w1;
          if (WREG) {
            w0 = (f32x4){wvh[0], wvh[1], wvh[2], wvh[3]};
            w1 = (f32x4){wvh[4], wvh[5], wvh[6], wvh[7]};
          } else {
            w0 = *(const f32x4*)(lds + L.Wv + 4 * hj);
            w1 = *(const f32x4*)(lds + L.Wv + 32 + 4 * hj);
          }
          vp = dot8(w0, w1, hc0, hc1);
        }
        if (!MH) vp = sum8(vp);
        const float v = vp + lds[L.bv];
        HEAD_STAMP(0);
        const float adv = sc[2], ret = sc[3];
        float logp = 0.f, ent = 0.f;
        float p[AMAX], lp[AMAX], xa[AMAX];
        if (CONT) {
          // sum_k [-(x-mu)^2 / (2 var) - log sigma - log sqrt(2 pi)] as
          // -sum_k (x-mu)^2 / (2 var) - sum_k (log sigma + log sqrt(2 pi)); 1/(2 var) is 0 for k >= A
          float q = 0.f;
#pragma unroll
          for (int k = 0; k < AMAX; ++k) {
            xa[k] = cact[k >> 2][k & 3];  // zero past A (record padding / unloaded chunks)
            const float d = xa[k] - out[k];
            q += (d * d) * lds[L.gc + k];
          }
          logp = -q - lds[L.gent + 1];
          ent = lds[L.gent];
        } else {
          const int actn = __float_as_int(sc[0]);
          float mx = out[0];
#pragma unroll
          for (int k = 1; k < AMAX; ++k)
            if (k < a.A) mx = fmaxf(mx, out[k]);
          float se = 0.f;
#pragma unroll
          for (int k = 0; k < AMAX; ++k)
            if (k < a.A) se += __expf(out[k] - mx);
          // se >= 1 (its largest term is exp(0)): the bare v_log_f32 (log2) needs no range fix-up
          const float lse = mx + __builtin_amdgcn_logf(se) * kLn2;
#pragma unroll
          for (int k = 0; k < AMAX; ++k) {
            lp[k] = out[k] - lse;
            p[k] = k < a.A ? __expf(lp[k]) : 0.f;  // p = 0 past A: no head delta, no entropy
            ent -= p[k] * lp[k];
            logp = k == actn ? lp[k] : logp;
          }
        }
        HEAD_STAMP(1);
        const float ratio = __expf(logp - sc[1]);                        // ppo.py:266
        const float rcl = fminf(fmaxf(ratio, 1.0f - a.clip_eps), 1.0f + a.clip_eps);
        const float u = -adv * ratio, w = -adv * rcl;                    // ppo.py:267-269
        const float inr = (ratio >= 1.0f - a.clip_eps && ratio <= 1.0f + a.clip_eps) ? 1.f : 0.f;
        const float gu = u > w ? 1.f : (u == w ? 0.5f : 0.f);            // torch.max splits ties
        const float gw = w > u ? 1.f : (u == w ? 0.5f : 0.f);
        const float vm = valid ? a.inv_m : 0.f;
        const float dlogp = (gu * -adv + gw * -adv * inr) * vm * ratio;
        const float dv = a.vf * (v - ret) * vm;                           // ppo.py:272
        if (valid && hj == 0) {
          s_pi += fmaxf(u, w);
          s_v += 0.5f * (v - ret) * (v - ret);
          s_ent += ent;
        }
        // DOUT[s] = {dout[0..A) | dv at 32 | dls at 33..}; the sample's 8 lanes split the writes
        float* drow = DOUT + hs * SD;
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
          if ((k & 7) == hj) {  // k >= A: zero deltas / log-std slots nobody reads
            float dk, dl = 0.f;
            if (CONT) {
              const float dd = xa[k] - out[k];
              const float z = dd * lds[L.gc + 32 + k];
              dk = dlogp * dd * lds[L.gc + 16 + k];
              dl = dlogp * (z * z - 1.0f);
            } else {
              const int actn = __float_as_int(sc[0]);
              dk = dlogp * ((k == actn ? 1.f : 0.f) - p[k]) + a.ent * vm * p[k] * (lp[k] + ent);
            }
            drow[k] = dk;
            if (CONT) drow[33 + k] = dl;
          }
        }
        if (hj == 0) drow[32] = dv;
        HEAD_STAMP(2);
      }
      // the next step's sample records (gathered in interval 5, heads of the next set) and the
      // index after that
      load_rec(it + 1);
      load_idx(it + 2);
      STEP_BARRIER();
      // ---- (5) head weight gradients (lane = feature column) and dZa, dZc of this wave's rows;
      // then the gather of step it+1 (its X0 buffer was last read by team 1 in interval 3)
      if (act) {
        constexpr int NA4D = (AMAX + 3) / 4;  // f32x4 chunks of a sample's head deltas
        constexpr int UNR = AMAX <= 4 ? SPW : 2;
#pragma unroll UNR
        for (int j = 0; j < SPW; ++j) {
          const int s = SPW * q + j;
          const float* drow = DOUT + s * SD;
          const float ha = HAC[s * SAC + lane];
          const float hc = HAC[s * SAC + 64 + lane];
#pragma unroll
          for (int c = 0; c < NA4D; ++c) {
            const f32x4 dk = *(const f32x4*)(drow + 4 * c);  // broadcast read
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (4 * c + e < AMAX) gWo[4 * c + e] += dk[e] * ha;  // rows >= A: zero deltas
          }
          gWv += drow[32] * hc;
          gbh += drow[lane];  // lanes < A: bo; lane 32: bv; lanes 33..: log-std terms
        }
        f32x4 dza[NSB], dzc[NSB], har[NSB], hcr[NSB];
        get_rows(har, HAC, SAC, row0, l15, h4);
        get_rows(hcr, HAC, SAC, 64 + row0, l15, h4);
#pragma unroll
        for (int sb = 0; sb < NSB; ++sb) {
          const float* drow = DOUT + (16 * sb + l15) * SD;
          const float dvs = drow[32];
          f32x4 dk[NA4D], dz = (f32x4){0.f, 0.f, 0.f, 0.f};
          if (MH) {
            // Wo^T dout on the matrix core: A = this wave's Wo columns, B = the sample's deltas
#pragma unroll
            for (int t = 0; t < 2; ++t) dz = mfma16(woT[t], drow[4 * t + h4], dz);
          } else {
#pragma unroll
            for (int c = 0; c < NA4D; ++c) dk[c] = *(const f32x4*)(drow + 4 * c);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = row0 + 4 * r + h4;  // perm(row0 + 4 h4 + r)
            float acc = 0.f;
            if (MH) {
              acc = dz[r];
            } else {
#pragma unroll
              for (int k = 0; k < AMAX; ++k)
                acc += (WREG ? wod[k < AR ? k : 0][r] : lds[L.Wo + k * H + col]) *
                       dk[k >> 2][k & 3];  // head-image rows >= A are zero
            }
            const float y = har[sb][r];
            dza[sb][r] = acc * (1.0f - y * y);
            const float yc = hcr[sb][r];
            dzc[sb][r] = (WREG ? wvd[r] : lds[L.Wv + col]) * dvs * (1.0f - yc * yc);
          }
          gba += dza[sb];
          gbc += dzc[sb];
        }
        put_rows(DZAC, SAC, row0, dza, l15, h4);
        put_rows(DZAC, SAC, 64 + row0, dzc, l15, h4);
      }
      gather(it + 1);
      csc = psc;
#pragma unroll
      for (int c = 0; c < NA4; ++c) cact[c] = pact[c];
      STEP_BARRIER();
    }

    EDGE_STAMP(2);
    // ---- epilogue (forward team): actor/critic hidden-bias rows into the slab image; head
    // partials and loss sums combined over the 4 waves through LDS in a fixed order
    zero_image(img, nimg4, tid);
    __syncthreads();  // (Z) the image is zero: padding floats stay zero in the slab
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float va = gba[r], vc = gbc[r];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        va += __shfl_xor(va, off);
        vc += __shfl_xor(vc, off);
      }
      if (l15 == 0) {
        img[po.ba + row0 + 4 * h4 + r] = va;
        img[po.bc + row0 + 4 * h4 + r] = vc;
      }
    }
    for (int off = 32; off >= 1; off >>= 1) {
      s_pi += __shfl_xor(s_pi, off);
      s_v += __shfl_xor(s_v, off);
      s_ent += __shfl_xor(s_ent, off);
    }
    constexpr int NH = AMAX + 3;
    float* hp = lds_ + q * NH * 64;  // the step images are dead (final barrier above)
#pragma unroll
    for (int k = 0; k < AMAX; ++k) hp[k * 64 + lane] = gWo[k];
    hp[AMAX * 64 + lane] = gWv;
    hp[(AMAX + 1) * 64 + lane] = gbh;
    hp[(AMAX + 2) * 64 + lane] = lane == 0 ? s_pi : (lane == 1 ? s_v : (lane == 2 ? s_ent : 0.f));
    // (R) rendezvous: team 1 joins this barrier after writing its accumulators into the image
    __syncthreads();
    const int c15 = lane & 15;
    const int ftrue = (lane & ~15) + 4 * (c15 & 3) + (c15 >> 2);  // true feature of column lane
    for (int e = q; e < NH; e += kTeamWaves) {
      const float v = ((lds_[(0 * NH + e) * 64 + lane] + lds_[(1 * NH + e) * 64 + lane]) +
                       lds_[(2 * NH + e) * 64 + lane]) + lds_[(3 * NH + e) * 64 + lane];
      if (e < AMAX) {
        if (e < a.A) img[po.Wo + e * H + ftrue] = v;
      } else if (e == AMAX) {
        img[po.Wv + ftrue] = v;
      } else if (e == AMAX + 1) {
        if (lane < a.A) img[po.bo + lane] = v;
        if (lane == 32) img[po.bv] = v;
        if (CONT && lane >= 33 && lane < 33 + a.A) img[po.ls + (lane - 33)] = v;
      } else {
        if (lane < 3) img[a.p_total + lane] = v;
      }
    }
  } else {
    // =========================== backward team ===========================
    float w2b[16], wab[16], wcb[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int k = 4 * t + h4;
      const int o = k * kStageRow + row0 + l15;
      w2b[t] = stg[o];
      wab[t] = stg[H * kStageRow + o];
      wcb[t] = stg[2 * H * kStageRow + o];
    }
    f32x4 gW1[2], gW2[4], gWa[4], gWc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gW2[i] = gWa[i] = gWc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (i < 2) gW1[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    f32x4 gb1 = (f32x4){0.f, 0.f, 0.f, 0.f}, gb2 = gb1;  // hidden-bias partials (b1, b2 rows)
    // (a static s_setprio 1 for this younger, MFMA-heavy half measured 3-4 % slower: the forward
    // team's VALU phases are the critical path)
    __syncthreads();  // LDS head weights / biases visible (pairs with team 0's)
#ifdef DPPO_PHASE_TRACE
    int tr_k_ = 0;
#endif

    for (int it = 0; it <= nit; ++it) {
      const bool act = it >= 1;  // works on step it-1
      const int b = (it + 1) & 1;
      float* lds = opaque_base(lds_);
      float* X0 = lds + L.X0[b];
      float* H1 = lds + L.H1[b];
      float* H2 = lds + L.H2[b];
      float* DZAC = lds + L.DZAC[b];
      float* DZ2 = lds + L.DZ2;
      float* DZ1 = lds + L.DZ1;
      // ---- (1) dh2 = Wa^T dZa + Wc^T dZc ; dZ2 = dh2 (1 - h2^2)
      if (act) {
        f32x4 dz2[NSB], h2r[NSB];
        zero(dz2);
        mm_rows<16>(dz2, wab, DZAC, SAC, l15, h4);
        mm_rows<16>(dz2, wcb, DZAC + 64, SAC, l15, h4);
        get_rows(h2r, H2, SA, row0, l15, h4);
#pragma unroll
        for (int sb = 0; sb < NSB; ++sb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dz2[sb][r] *= (1.0f - h2r[sb][r] * h2r[sb][r]);
          gb2 += dz2[sb];
        }
        put_rows(DZ2, SA, row0, dz2, l15, h4);
      }
      STEP_BARRIER();
      // ---- (2) dh1 = W2^T dZ2 ; dZ1 = dh1 (1 - h1^2)
      if (act) {
        f32x4 dz1[NSB], h1r[NSB];
        zero(dz1);
        mm_rows<16>(dz1, w2b, DZ2, SA, l15, h4);
        get_rows(h1r, H1, SA, row0, l15, h4);
#pragma unroll
        for (int sb = 0; sb < NSB; ++sb) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dz1[sb][r] *= (1.0f - h1r[sb][r] * h1r[sb][r]);
          gb1 += dz1[sb];
        }
        put_rows(DZ1, SA, row0, dz1, l15, h4);
      }
      STEP_BARRIER();
      // ---- (3) dW1 += dZ1 X0^T only: team 0 runs its MFMA-heavy actor / critic layers here
      // (dW1 cannot move later: team 0 gathers the next step into this X0 buffer in interval 5)
      if (act) {
        if (nk1 == 8) wgrad16<2>(gW1, DZ1, SA, 0, X0, SX0, 0, row0, l15, h4);
        else wgrad16<1>(gW1, DZ1, SA, 0, X0, SX0, 0, row0, l15, h4);
      }
      STEP_BARRIER();
      // ---- (4) dWa += dZa H2^T ; dW2 += dZ2 H1^T  (team 0: heads + loss on VALU)
      if (act) {
        wgrad16<4>(gWa, DZAC, SAC, 0, H2, SA, 0, row0, l15, h4);
        wgrad16<4>(gW2, DZ2, SA, 0, H1, SA, 0, row0, l15, h4);
      }
      STEP_BARRIER();
      // ---- (5) dWc += dZc H2^T  (team 0: head back-propagation on VALU)
      if (act) wgrad16<4>(gWc, DZAC, SAC, 64, H2, SA, 0, row0, l15, h4);
      STEP_BARRIER();
    }

    // ---- epilogue (backward team): each wave owns distinct rows of dW1, dW2, dWa, dWc, b1, b2
    zero_image(img, nimg4, tid);
    __syncthreads();  // (Z) pairs with the forward team's
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = row0 + 4 * h4 + r;
#pragma unroll
      for (int ib = 0; ib < 4; ++ib) {
        const int i = 16 * ib + l15;
        img[po.W2 + o * H + i] = gW2[ib][r];
        img[po.Wa + o * H + i] = gWa[ib][r];
        img[po.Wc + o * H + i] = gWc[ib][r];
      }
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const int i = 16 * ib + l15;
        if (i < a.D) img[po.W1 + o * a.D + i] = gW1[ib][r];
      }
      float v1 = gb1[r], v2 = gb2[r];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        v1 += __shfl_xor(v1, off);
        v2 += __shfl_xor(v2, off);
      }
      if (l15 == 0) {
        img[po.b1 + o] = v1;
        img[po.b2 + o] = v2;
      }
    }
    __syncthreads();  // (R) pairs with the forward team's head-partial rendezvous
  }
  // the assembled slab leaves as 16-B write-through stores: ~13 MB per launch over the whole chip
  // while the kernel drains, instead of 4-B pieces or dirty lines at the kernel boundary
  __syncthreads();
  for (int c = tid; c < nimg4; c += kThreads) slab_put4(slab + 4 * c, ((const f32x4*)img)[c]);
#ifdef DPPO_PHASE_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  EDGE_STAMP(3);
  EDGE_REAL(5);
#endif
  if (a.fuse) fused_reduce_adam(a, lds_);
}

}  // namespace

#ifdef DPPO_PHASE_TRACE
extern "C" __attribute__((visibility("default"))) int dppo_debug_phase_trace(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_trace), sizeof(g_phase_trace)) == hipSuccess
             ? 0
             : -2;
}
extern "C" __attribute__((visibility("default"))) int dppo_debug_phase_edges(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_edges), sizeof(g_phase_edges)) == hipSuccess
             ? 0
             : -2;
}
extern "C" __attribute__((visibility("default"))) int dppo_debug_heads_trace(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_heads_trace), sizeof(g_heads_trace)) == hipSuccess
             ? 0
             : -2;
}
#endif

size_t mb_lds_bytes(const MlpShape& sh) {
  const int D16 = (sh.D + 15) / 16 * 16;
  const Lds2 L = make_lds2(D16);
  const int stage = L.H1[0] + kStageFloats;  // prologue weight staging over the step images
  return (size_t)(L.total > stage ? L.total : stage) * sizeof(float);
}

int mb_grid(const MlpShape& sh, int32_t m, bool fused) {
  if (!fused && mbw_supported(sh)) return mbw_grid(m);
  const int nsteps = (m + S - 1) / S;
  int g = nsteps;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  return g;
}

int launch_mb(const MlpShape& sh, const ParamOffsets& po, const GradArgs& ga, int G,
              hipStream_t s, const FusedAdam* fused) {
  if (!fused && mbw_supported(sh)) return launch_mbw(sh, po, ga, G, s);
  MArgs k{};
  const int D16 = (sh.D + 15) / 16 * 16;
  k.L = make_lds2(D16);
  k.po = po;
  k.params = ga.params;
  k.rec = ga.rec;
  k.idx = ga.idx;
  k.seg = ga.seg;
  k.m = ga.m;
  k.inv_m = ga.inv_m;
  k.clip_eps = ga.clip_eps;
  k.vf = ga.vf_coef;
  k.ent = ga.ent_coef;
  k.slabs = ga.slabs;
  k.slab_stride = ga.slab_stride;
  k.p_total = ga.p_total;
  k.D = sh.D;
  k.D8 = sh.D8;
  k.D16 = D16;
  k.A = sh.A;
  k.R = sh.R;
  if (fused) {
    k.fuse = 1;
    k.fa = *fused;
    k.nblk = (int)((ga.p_total + 8 + kTailParams - 1) / kTailParams);
  }
  size_t lds = (size_t)k.L.total * sizeof(float);
  // the prologue stages W2 | Wa | Wc over the step images; the epilogue reuses them for the
  // per-wave head partials and the workgroup's slab image
  const size_t stage = (size_t)(k.L.H1[0] + kStageFloats) * sizeof(float);
  const size_t epi = (size_t)(kEpiHead + (ga.p_total + 8 + 3) / 4 * 4) * sizeof(float);
  if (stage > lds) lds = stage;
  if (epi > lds) lds = epi;
  if (lds > 160 * 1024) {
    set_error("fused minibatch kernel needs %zu bytes of LDS (> 160 KiB)", lds);
    return DPPO_EUNSUPPORTED;
  }
  static const bool attr = [] {
#define DPPO_SET2(A, C) raise_dyn_lds((const void*)mb_kernel<A, C>);
    DPPO_SET2(2, false) DPPO_SET2(2, true) DPPO_SET2(4, false) DPPO_SET2(4, true)
    DPPO_SET2(8, false) DPPO_SET2(8, true) DPPO_SET2(16, false) DPPO_SET2(16, true)
#undef DPPO_SET2
    return true;
  }();
  (void)attr;
  const dim3 grid((unsigned)G), block(kThreads);
  const bool c = sh.continuous != 0;
  if (sh.A <= 2) {
    if (c) DPPO_LAUNCH((mb_kernel<2, true>), grid, block, lds, s, k);
    else DPPO_LAUNCH((mb_kernel<2, false>), grid, block, lds, s, k);
  } else if (sh.A <= 4) {
    if (c) DPPO_LAUNCH((mb_kernel<4, true>), grid, block, lds, s, k);
    else DPPO_LAUNCH((mb_kernel<4, false>), grid, block, lds, s, k);
  } else if (sh.A <= 8) {
    if (c) DPPO_LAUNCH((mb_kernel<8, true>), grid, block, lds, s, k);
    else DPPO_LAUNCH((mb_kernel<8, false>), grid, block, lds, s, k);
  } else {
    if (c) DPPO_LAUNCH((mb_kernel<16, true>), grid, block, lds, s, k);
    else DPPO_LAUNCH((mb_kernel<16, false>), grid, block, lds, s, k);
  }
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
