// Fused PPO minibatch step, sample-split form: one wave per SIMD, and each wave runs the whole
// gather -> forward -> loss -> analytic backward -> weight-gradient accumulation of its own
// 16-sample groups with every activation in registers.  No workgroup barrier inside the main
// loop: the only cross-wave step is the final sum of the four waves' gradients.
//
// Reference: loss and backward of one minibatch, diamond/ppo.py:261-283 (continuous:
// continuous_ppo.py:273-295), default networks ppo.py:53-71 / continuous_ppo.py:63-81.
//
// ---- Register layouts (lane l = 16 q + r of a wave) --------------------------------------------
// v_mfma_f32_16x16x4_f32 takes A[i][k] from lane (q = k, r = i), B[k][j] from lane (k, j) and
// leaves D[4q + v][r] in register v of lane (q, r).
// * N layout of a [64 features x 16 samples] activation, four f32x4 tiles b: register v of tile b
//   in lane (q, r) = feature 16b + 4q + v of sample r.  It is what the forward produces (A =
//   weight rows, B = input) and, read as B with k-step (b, v) <-> features {16b + 4q + v}, what
//   the next layer consumes: the forward chains in registers.
// * P layout: register v of tile b in lane (q, r) = feature 4r + b of sample 4q + v.  The
//   backward produces it (A = dZ in N layout, i.e. i = sample; B = one ds_read_b128 of the row
//   W[out][4r .. 4r + 3], whose four floats feed the four output tiles b) and the weight gradient
//   dW += dZ X^T takes both operands in it (k = sample, k-step v <-> samples {4q + v}); the
//   accumulated dW tiles come out feature-permuted and are put back in order by the epilogue.
// Each layer therefore needs its input activation and its output delta in both layouts; the
// N <-> P turns go through a wave-private LDS scratch of sample-major rows (stride 68), 16-B
// reads and writes both ways.
//
// ---- LDS ------------------------------------------------------------------------------------------
// The hidden weights W2, Wa, Wc stay in LDS for the launch (read-only), rows padded to 68 floats:
// the forward's row-slice ds_read_b128 (lane (q, r): row 16ob + r, floats 16kb + 4q ..) and the
// backward's column ds_read_b32 (lane (q, r): row 16ob + 4q + v, column 16rb + r) both address
// one base register per lane plus compile-time offsets (the layout is constexpr), and are
// conflict-free (b32) / one 2-way pair per 16-lane group (b128).
//
// Heads (at most 4 actions) and the per-sample loss run on VALU in the N layout: each lane dots
// the 16 head-input features it holds, the four lanes of a sample (q = 0..3) are summed with
// v_permlane16/32_swap, and every lane then has its sample's logits / mean and value.
//
// Every partial sum is reduced in a fixed order and written once per workgroup into its gradient
// slab (optim.hip sums the slabs in a fixed order): bit-reproducible, no float atomics.
#include "common.h"

namespace dppo {
namespace {

constexpr int H = 64;
constexpr int kWavesW = 4;                  // one wave per SIMD
constexpr int kThreadsW = kWavesW * kWave;  // 256
constexpr int kSm = 68;                     // turn scratch: [16 samples][68]
constexpr int kSlot = 16 * kSm;                       // one turn slot
constexpr int kSdw = 12;                              // head-delta row: dlogit[8] | dvalue
constexpr int kScratch = 4 * kSlot + 16 * kSdw;       // floats per wave: 4 slots + head deltas
constexpr int kMat = H * H;                 // one hidden weight matrix
constexpr float kLogSqrt2PiW = 0.91893853320467274178f;
constexpr float kLn2W = 0.69314718055994530942f;
constexpr float kHalfLog2PiPlusHalfW = 1.41893853320467274178f;

// Scheduling fence between the phases of a group: keeps the compiler from hoisting one phase's
// LDS / global loads into the previous one (which raises register pressure past the budget of
// one wave per SIMD: 208 accumulator + ~230 working registers).
#define PHASE_FENCE() __builtin_amdgcn_sched_barrier(0)

#ifdef DPPO_PHASE_TRACE
// per workgroup: s_memtime at entry, main-loop entry, main-loop exit, end; s_memrealtime at entry
// and at the end (in-kernel clock, cross-CU skew)
__device__ long long g_mbw_edges[256][6];
#define WEDGE(i, v)                                                     \
  do {                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 256) g_mbw_edges[blockIdx.x][i] = (v); \
  } while (0)
// workgroup 0: s_memtime of every wave at each phase fence of its first 16 groups
constexpr int kTrGroups = 16, kTrPhases = 10;
__device__ long long g_mbw_phase[kWavesW][kTrGroups][kTrPhases];
// workgroup 0, thread 0: s_memtime at the steps of the epilogue
__device__ long long g_mbw_epi[8];
#define ESTAMP(i)                                                                        \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_mbw_epi[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define WSTAMP(k, i)                                                                     \
  do {                                                                                   \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (k) < kTrGroups)                   \
      g_mbw_phase[threadIdx.x >> 6][(k)][(i)] = __builtin_amdgcn_s_memtime();            \
  } while (0)
#else
#define WSTAMP(k, i) \
  do {               \
  } while (0)
#define ESTAMP(i) \
  do {            \
  } while (0)
#define WEDGE(i, v) \
  do {              \
  } while (0)
#endif

constexpr int kWS = 68;  // row stride of the hidden weight images

struct WLds {   // offsets in floats (compile-time: one layout per input width)
  int W2;       // W2 | Wa | Wc: [3][64][kWS]
  int scratch;  // [4 waves][kScratch]
  int Wo, Wv;   // [8][64] (rows >= A zero), [64]
  int b1, b2, ba, bc;
  int bo, bv, ls;  // [8], [4], [8]
  int gc;       // [4][8]: 1/(2 var), 1/var, 1/sigma, log sigma per action (continuous)
  int gent;     // [4]: {sum entropy terms, sum log-prob constants}
  int W1, RS1;  // W1 image [64 rows][RS1 >= D16], k-step-major per lane (layer1_w1)
  int total;
};

struct WArgs {
  ParamOffsets po;
  const float* params;
  const float* rec;
  const int32_t* idx;
  const int32_t* seg;  // global-minibatch DP: {start, end} of this minibatch in idx (device)
  int m;
  float inv_m, clip_eps, vf, ent;
  float* slabs;
  int64_t slab_stride, p_total;
  int D, D8, A, R, nkn;
  int plain_slab;  // DPPO_SLAB_PLAIN=1 (A/B): plain slab stores (L2-resident, written back at the
                   // kernel boundary) instead of write-through
};

constexpr WLds make_wlds(int D16) {
  WLds L{};
  int o = 0;
  L.W2 = o;
  o += 3 * H * kWS;
  L.scratch = o;
  o += kWavesW * kScratch;
  L.Wo = o;
  o += 8 * H;
  L.Wv = o;
  o += H;
  L.b1 = o;
  o += H;
  L.b2 = o;
  o += H;
  L.ba = o;
  o += H;
  L.bc = o;
  o += H;
  L.bo = o;
  o += 8;
  L.bv = o;
  o += 4;
  L.ls = o;
  o += 8;
  L.gc = o;
  o += 32;
  L.gent = o;
  o += 4;
  L.W1 = o;
  L.RS1 = D16 + 2;
  o += H * L.RS1;
  L.total = (o + 3) & ~3;
  return L;
}

// Epilogue staging: two [4 waves][64 x 64] buffers, then the small per-wave items
// {biases b1 b2 ba bc | AMAX head rows | Wv | 2 AMAX + 4 scalars}.
constexpr int small_floats(int amax) { return (5 + amax) * H + 2 * amax + 4; }
constexpr int epi_floats(int amax) {
  return 2 * kWavesW * kMat + kWavesW * ((small_floats(amax) + 3) & ~3);
}

// Instruction-group pins for the scheduler (llvm.amdgcn.sched.group.barrier): under the register
// pressure of one wave per SIMD it otherwise re-uses one operand buffer and waits on every LDS read
// right before its MFMAs.  Masks: MFMA 0x8, DS read 0x100.
#define SG_MFMA(n) __builtin_amdgcn_sched_group_barrier(0x008, (n), 0)
#define SG_DSR(n) __builtin_amdgcn_sched_group_barrier(0x100, (n), 0)
#define SG_VALU(n) __builtin_amdgcn_sched_group_barrier(0x002, (n), 0)
#define SG_DSW(n) __builtin_amdgcn_sched_group_barrier(0x200, (n), 0)
#define SG_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The weight-gradient accumulation in AGPR form (accumulator read and written in place in the
// AGPRs) while the rest of the file builds in VGPR form: the gradient tiles live in AGPRs across
// the whole loop, and a VGPR-form MFMA on them needed them copied into VGPRs and back (the loop
// of the CartPole instantiation: 326 AGPR reads -> 28).  Measured per launch: C2 55.5 -> 54.5 µs,
// C3 100.9 -> 99.6; the Gaussian-head instantiations measured slower (C4 63.1 -> 64.6) and keep
// the builtin.  DPPO_MBW_VGPR_WGRAD: the builtin everywhere (A/B).
template <bool AGPR>
__device__ __forceinline__ void mfma4_acc(float a, float b, f32x4& c) {
#ifndef DPPO_MBW_VGPR_WGRAD
  if constexpr (AGPR) {
    asm("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
    return;
  }
#endif
  c = mfma4(a, b, c);
}

// ---- Packed fp32 (VOP3P) element-wise steps: two elements per instruction at the issue cost of
// one scalar VALU instruction, beside the fp32 MFMAs as alone (tools/probe/mfma_kind.py: v_fma_f32
// and v_pk_fma_f32 both ~5 cycles per instruction), on the two 64-bit halves of an f32x4 (aligned
// register pairs, no moves).  The compiler's own packing (the SLP vectorizer) paired elements of
// different tiles and paid a v_mov / v_xor per pair.
__device__ __forceinline__ f32x2 lo2(f32x4 v) { return __builtin_shufflevector(v, v, 0, 1); }
__device__ __forceinline__ f32x2 hi2(f32x4 v) { return __builtin_shufflevector(v, v, 2, 3); }
__device__ __forceinline__ f32x4 cat2(f32x2 a, f32x2 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3); }
// (compiler vector code: this file builds with packed fp32 on and the SLP vectorizer off, so only
// these explicit f32x2 operations become packed instructions, and the hazard recognizer sees
// them -- an inline-asm form failed the audit of tools/mfma_hazards.py, rules R4-R7)
__device__ __forceinline__ f32x2 pk_mul(f32x2 a, f32x2 b) { return a * b; }
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(a, b, c);
}
template <int S>
__device__ __forceinline__ f32x2 pk_fma_bc(f32x2 a, f32x2 s, f32x2 c) {
  return __builtin_elementwise_fma(a, __builtin_shufflevector(s, s, S, S), c);
}
template <int S>
__device__ __forceinline__ f32x2 pk_mul_bc(f32x2 a, f32x2 s) {
  return a * __builtin_shufflevector(s, s, S, S);
}
__device__ __forceinline__ f32x2 pk_add1(f32x2 e) { return e + 1.0f; }
__device__ __forceinline__ f32x2 pk_one_m2(f32x2 r) {
  return __builtin_elementwise_fma((f32x2)(-2.0f), r, (f32x2)(1.0f));
}
__device__ __forceinline__ f32x2 pk_dtanh(f32x2 dy, f32x2 y) {
  return dy * __builtin_elementwise_fma(-y, y, (f32x2)(1.0f));
}
__device__ __forceinline__ f32x4 dtanh4(f32x4 dy, f32x4 y) {
  return cat2(pk_dtanh(lo2(dy), lo2(y)), pk_dtanh(hi2(dy), hi2(y)));
}
// sum_k w[k] x[k] over four f32x4 of 16 elements: 8 packed instructions in two independent
// chains (low and high halves) + 2 adds.  (One chain of 8: each packed FMA waited for the one
// before it, with a wait state between dependent packed instructions on top.)
__device__ __forceinline__ float pk_dot16(const f32x4 (&w)[4], const f32x4 (&x)[4]) {
  f32x2 pa = pk_mul(lo2(w[0]), lo2(x[0]));
  f32x2 pb = pk_mul(hi2(w[0]), hi2(x[0]));
#pragma unroll
  for (int b = 1; b < 4; ++b) {
    pa = pk_fma(lo2(w[b]), lo2(x[b]), pa);
    pb = pk_fma(hi2(w[b]), hi2(x[b]), pb);
  }
  const f32x2 p = pa + pb;
  return p[0] + p[1];
}

__device__ __forceinline__ float tanh_w(float x) {
  // tanh = 1 - 2 / (e^{2x} + 1): five instructions (v_exp, v_rcp and three plain ones) beside a
  // wave's MFMAs; saturates to +-1 through e^{2x} = inf / 0, absolute error <= ~1.2e-7 (the
  // cancellation near 0 costs relative, not absolute, accuracy, as in every exp-based form)
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2 log2(e)
  return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

// The hidden layers' weights and biases are staged into LDS pre-multiplied by kTS = 2 log2(e),
// so a layer's MFMAs produce kTS z directly and its tanh needs no multiply (4 VALU instructions
// per activation instead of 5: on gfx950 fp32 MFMA work every VALU instruction costs its issue
// slot).  The backward pass runs through the same scaled images: dh2 comes out
// kTS-scaled and dh1 kTS^2-scaled, so the W2 / b2 gradients carry kTS and W1 / b1 kTS^2, undone
// once per launch in the epilogue (a few ulp against the unscaled products; the parity bounds
// are 2e-5 of the gradient scale).
constexpr float kTS = 2.8853900817779268f;
constexpr float kInvTS = 1.0f / kTS;
constexpr float kInvTS2 = 1.0f / (kTS * kTS);

// Sixteen activations stage by stage (all exps, all adds, ...) from pre-scaled inputs kTS z:
// consecutive instructions are independent, so that pinned between MFMAs each issue slot holds
// work that is ready.
// The two plain steps as packed instructions (two elements each, above).
__device__ __forceinline__ void tanh4(f32x4 (&y)[4]) {
  f32x4 e[4];
#pragma unroll
  for (int i = 0; i < 16; ++i) e[i >> 2][i & 3] = __builtin_amdgcn_exp2f(y[i >> 2][i & 3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = cat2(pk_add1(lo2(e[i])), pk_add1(hi2(e[i])));
#pragma unroll
  for (int i = 0; i < 16; ++i) e[i >> 2][i & 3] = __builtin_amdgcn_rcpf(e[i >> 2][i & 3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = cat2(pk_one_m2(lo2(e[i])), pk_one_m2(hi2(e[i])));
}

// Sum over the four lanes of a sample (q = 0..3, same r): rows 0+1 and 2+3 with
// v_permlane16_swap, then the two halves with v_permlane32_swap.  The same additions in the same
// order in every lane.
__device__ __forceinline__ float qsum(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  const float s = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto p2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false,
                                                   false);
  return __uint_as_float(p2[0]) + __uint_as_float(p2[1]);
}

// Sum over each 16-lane row (the result in every lane of the row) with DPP lane moves: lane ^ 1,
// lane ^ 2, the mirrored half-row, the mirrored row.
template <int CTRL>
__device__ __forceinline__ float dppw(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16(float x) {
  x += dppw<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dppw<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dppw<0x141>(x);  // row_half_mirror
  x += dppw<0x140>(x);  // row_mirror
  return x;
}

__device__ __forceinline__ float dot4(f32x4 w, f32x4 x) {
  return (w[0] * x[0] + w[1] * x[1]) + (w[2] * x[2] + w[3] * x[3]);
}

// DPPO_ABL_NOCONFLICT (timing-only ablation, wrong results): the hidden-weight and scratch
// ds_read_b128 of the main loop read addresses that keep every lane group on distinct banks
// (lanes with the same r read the same 16 B), to bound what the 2-way conflicts of the real
// layout cost.
#ifdef DPPO_ABL_NOCONFLICT
#define ABL_FWD(q, r) (4 * (r))
#define ABL_BWD(q, r) (4 * (r))
#else
#define ABL_FWD(q, r) ((r) * kWS + 4 * (q))
#define ABL_BWD(q, r) (4 * (q) * kWS + 4 * (r))
#endif

// Forward of one hidden layer, N -> N: y[ob] += W[16ob + i][:] x for the four 16-row output
// blocks; the A operand of k-steps (kb, 0..3) is one ds_read_b128 of the row.
// The A operands of k-block 0 (fwd64_first), read by the caller ahead of the layer or here.
__device__ __forceinline__ void fwd64_first(f32x4 (&w0)[4], const float* W, int q, int r) {
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) w0[ob] = *(const f32x4*)(W + 16 * ob * kWS + ABL_FWD(q, r));
}
__device__ __forceinline__ void fwd64_pre(f32x4 (&y)[4], const float* W, const f32x4 (&x)[4],
                                          int q, int r, const f32x4 (&w0)[4]) {
  f32x4 w[2][4];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) w[0][ob] = w0[ob];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb + 1 < 4) {
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
        w[(kb + 1) & 1][ob] = *(const f32x4*)(W + 16 * ob * kWS + 16 * (kb + 1) + ABL_FWD(q, r));
    }
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) y[ob] = mfma4(w[kb & 1][ob][v], x[kb][v], y[ob]);
  }
}
__device__ __forceinline__ void fwd64_raw(f32x4 (&y)[4], const float* W, const f32x4 (&x)[4],
                                          int q, int r) {
  f32x4 w0[4];
  fwd64_first(w0, W, q, r);
  fwd64_pre(y, W, x, q, r, w0);
}
__device__ __forceinline__ void fwd64(f32x4 (&y)[4], const float* W, const f32x4 (&x)[4], int q,
                                      int r) {
  SG_FENCE();
  fwd64_raw(y, W, x, q, r);
  // the next k-block's four row reads go out among this block's 16 MFMAs
  SG_DSR(4);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (kb < 3) SG_DSR(1);
      SG_MFMA(4);
    }
  SG_FENCE();
}

// Two layers on the same input (actor / critic hidden): eight independent accumulation chains.
__device__ __forceinline__ void fwd64x2(f32x4 (&y)[4], const float* W, f32x4 (&z)[4],
                                        const float* U, const f32x4 (&x)[4], int q, int r) {
  SG_FENCE();
  f32x4 w[2][4], u[2][4];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o = 16 * ob * kWS + ABL_FWD(q, r);
    w[0][ob] = *(const f32x4*)(W + o);
    u[0][ob] = *(const f32x4*)(U + o);
  }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    if (kb + 1 < 4) {
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) {
        const int o = 16 * ob * kWS + 16 * (kb + 1) + ABL_FWD(q, r);
        w[(kb + 1) & 1][ob] = *(const f32x4*)(W + o);
        u[(kb + 1) & 1][ob] = *(const f32x4*)(U + o);
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) {
        y[ob] = mfma4(w[kb & 1][ob][v], x[kb][v], y[ob]);
        z[ob] = mfma4(u[kb & 1][ob][v], x[kb][v], z[ob]);
      }
  }
  SG_DSR(8);
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (kb < 3) SG_DSR(1);
      SG_MFMA(4);
    }
  SG_FENCE();
}

// Backward through one hidden layer into the P layout: t[b] += sum_out dz[out][s] W[out][4r + b]
// (A = dz in N layout; B = W[out][4r .. 4r + 3], one ds_read_b128 per k-step for all four tiles).
__device__ __forceinline__ void bwdP(f32x4 (&t)[4], const float* W, const f32x4 (&dz)[4], int q,
                                     int r) {
  SG_FENCE();
  f32x4 b[3];
  auto ld = [&](int k) {
    return *(const f32x4*)(W + (16 * (k >> 2) + (k & 3)) * kWS + ABL_BWD(q, r));
  };
  b[0] = ld(0);
  b[1] = ld(1);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k + 2 < 16) b[(k + 2) % 3] = ld(k + 2);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) t[rb] = mfma4(dz[k >> 2][k & 3], b[k % 3][rb], t[rb]);
  }
  // reads two k-steps ahead of their MFMAs
  SG_DSR(2);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k + 2 < 16) SG_DSR(1);
    SG_MFMA(4);
  }
  SG_FENCE();
}

// bwdP of two matrices into the same tiles (t += W^T dz + U^T du) as ONE 32-k-step pipeline: the
// second matrix's first rows are read during the first one's last k-steps instead of in a
// pipeline restart whose first MFMAs wait for their reads.
// The B operands of the first two k-steps (pre[0..1], bwdP_row(W, 0 / 1)) are read by the caller
// one phase early, so that the pipeline's first MFMAs do not wait for them.
__device__ __forceinline__ f32x4 bwdP_row(const float* W, int k, int q, int r) {
  return *(const f32x4*)(W + (16 * (k >> 2) + (k & 3)) * kWS + ABL_BWD(q, r));
}
__device__ __forceinline__ void bwdP2(f32x4 (&t)[4], const float* W, const f32x4 (&dz)[4],
                                      const float* U, const f32x4 (&du)[4], int q, int r,
                                      const f32x4 (&pre)[2]) {
  SG_FENCE();
  f32x4 b[3];
  auto ld = [&](int k) { return bwdP_row(k < 16 ? W : U, k & 15, q, r); };
  b[0] = pre[0];
  b[1] = pre[1];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k + 2 < 32) b[(k + 2) % 3] = ld(k + 2);
    const int kk = k & 15;
    const float av = k < 16 ? dz[kk >> 2][kk & 3] : du[kk >> 2][kk & 3];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) t[rb] = mfma4(av, b[k % 3][rb], t[rb]);
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k + 2 < 32) SG_DSR(1);
    SG_MFMA(4);
  }
  SG_FENCE();
}

// dW tiles += dZ X^T over the group's 16 samples (both operands in P layout, or X in the natural
// T layout of the input features for dW1).
template <int NIB, bool AGPR>
__device__ __forceinline__ void wgrad(f32x4* acc, const f32x4 (&dzt)[4], const f32x4* xt) {
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int ib = 0; ib < NIB; ++ib)
        mfma4_acc<AGPR>(dzt[ob][v], xt[ib][v], acc[ob * NIB + ib]);
}

// N -> P through the wave's scratch (sample-major rows of kSm floats): 16-B writes of the N tiles,
// 16-B reads of four P-layout registers (the four tiles of one sample 4q + v) each.
__device__ __forceinline__ void put_n(float* sm, const f32x4 (&n)[4], int q, int r) {
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) *(f32x4*)(sm + r * kSm + 16 * ob + 4 * q) = n[ob];
}
// The same reads without the renaming: x[v][b] = t[b][v] (x[v] is one loaded 16-B quad, an
// aligned register tuple that packed instructions can take by halves).
__device__ __forceinline__ void get_p_raw(f32x4 (&x)[4], const float* sm, int q, int r) {
#pragma unroll
  for (int v = 0; v < 4; ++v) x[v] = *(const f32x4*)(sm + (4 * q + v) * kSm + 4 * r);
}
// the loaded quad v behind a get_p result: (t[0][v], t[1][v], t[2][v], t[3][v]) -- the same
// registers, no data movement
__device__ __forceinline__ f32x4 quad_of(const f32x4 (&t)[4], int v) {
  return (f32x4){t[0][v], t[1][v], t[2][v], t[3][v]};
}
__device__ __forceinline__ void get_p(f32x4 (&t)[4], const float* sm, int q, int r) {
#pragma unroll
  for (int v = 0; v < 4; ++v) {
#ifdef DPPO_ABL_NOCONFLICT
    const f32x4 x = *(const f32x4*)(sm + v * kSm + 4 * r);
#else
    const f32x4 x = *(const f32x4*)(sm + (4 * q + v) * kSm + 4 * r);
#endif
#pragma unroll
    for (int b = 0; b < 4; ++b) t[b][v] = x[b];
  }
}
// P -> N.
__device__ __forceinline__ void put_p(float* sm, const f32x4 (&t)[4], int q, int r) {
#pragma unroll
  for (int v = 0; v < 4; ++v)
    *(f32x4*)(sm + (4 * q + v) * kSm + 4 * r) = (f32x4){t[0][v], t[1][v], t[2][v], t[3][v]};
}
__device__ __forceinline__ void get_n(f32x4 (&n)[4], const float* sm, int q, int r) {
#pragma unroll
#ifdef DPPO_ABL_NOCONFLICT
  for (int ob = 0; ob < 4; ++ob) n[ob] = *(const f32x4*)(sm + 16 * ob + 4 * r);
#else
  for (int ob = 0; ob < 4; ++ob) n[ob] = *(const f32x4*)(sm + r * kSm + 16 * ob + 4 * q);
#endif
}

__device__ __forceinline__ void slab_st4(float* p, f32x4 v) {
  // s_nop: a VALU write to the data VGPRs of a store wider than 8 bytes needs a wait state
  // after it, which the compiler cannot insert behind an asm statement (seen: back-to-back slab
  // stores whose next operands overwrote this one's data before it was read)
#if defined(DPPO_SLAB_NT_SC1)  // (A/B) the non-temporal cache policy on top
  asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#elif defined(DPPO_SLAB_NT)  // (A/B) non-temporal instead of write-through
  asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#else
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
#endif
}

__device__ __forceinline__ f32x4 z4() { return (f32x4){0.f, 0.f, 0.f, 0.f}; }

// One group's sample indices: the lane's own sample (N layout) and the four of the T layout.
struct Fetch {
  int sn, st[4];
};
// One group's record data.
template <int NIB>
struct GRec {
  float xn[4 * NIB];  // layer-1 B operand: input 4t + q of sample r
  f32x4 xt[NIB];      // T layout of the input: feature 16ib + r of samples 4q + v
  f32x4 sc;           // {action bits, old log-prob, advantage, return} of sample r
  f32x4 ca[2];        // continuous action of sample r (<= 8 dims)
  int sn;             // sample r's record (kLateCa: the action is read in the group's phase 3)
};

// Which instantiations hold the head rows in registers from the critic layer to the head
// back-propagation: up to 4 heads (spill-free; with 6-8 heads ROCm 7.2's compiler crashes in
// register allocation).  -DDPPO_MBW_PREHEADS=0 turns it off (A/B builds).
#ifndef DPPO_MBW_PREHEADS
#define DPPO_MBW_PREHEADS 1
#endif
template <int AMAX, bool CONT, int NIB>
constexpr bool kPreloadHeads() {
  return DPPO_MBW_PREHEADS && AMAX <= 4;
}

// X1: exactly 17 inputs (HalfCheetah).  Input column 16 is the only live one of the second
// 16-column block, so its dW1 column is a VALU rank-1 sum (16 FMAs per group) instead of four
// 16x16 MFMA tiles (16 MFMAs and 16 accumulator registers per group) -- the registers that
// made this instantiation spill.
template <int AMAX, bool CONT, int NIB, bool X1 = false>
__global__ __launch_bounds__(kThreadsW, 1) void mbw_kernel(WArgs a) {
  static_assert(!X1 || NIB == 2, "X1 is the 17-input layout");
  extern __shared__ __attribute__((aligned(16))) float lds[];
#ifdef DPPO_PHASE_TRACE
  // (timing-only build: only the instantiations tools/mbw_trace.py runs -- CartPole, LunarLander,
  // HalfCheetah; with the stamps in, the others crash ROCm 7.2's AGPR-copy rewrite pass)
  if constexpr (!((AMAX == 2 && !CONT && NIB == 1) || (AMAX == 4 && !CONT && NIB == 1) ||
                  (AMAX == 6 && CONT && X1)))
    return;
  WEDGE(0, (long long)__builtin_amdgcn_s_memtime());
  WEDGE(4, (long long)__builtin_amdgcn_s_memrealtime());
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, r = lane & 15;
  constexpr WLds L = make_wlds(16 * NIB);
  const float* P = a.params;
  const ParamOffsets& po = a.po;
  int mm = a.m;
  const int32_t* idxp = a.idx;
  if (a.seg) {  // this rank's share of a global minibatch is known only on the device
    const int s0 = a.seg[0];
    mm = a.seg[1] - s0;
    idxp += s0;
  }
  const int ngroups = (mm + 15) >> 4;
  const int first = (int)blockIdx.x * kWavesW + wave;  // group k of this wave: first + k * stride
  const int stride = (int)gridDim.x * kWavesW;
  const int nk = first < ngroups ? (ngroups - first + stride - 1) / stride : 0;
  const int R = a.R, D = a.D;
  // 5-8 Gaussian actions: the action is loaded at the start of its group's head layers instead
  // of a group ahead (8 registers fewer across the backward phases, where this kernel spills)
  constexpr bool kLateCa = CONT && (AMAX > 4 || NIB == 2);
  // ... and the T-layout input for dW1 (indices and records) is read in the group's own phase 7,
  // ~12 K cycles before its use, instead of being carried from the previous group
  constexpr bool kLateXt = kLateCa;
  // ... and the head-weight gradient is an MFMA tile sum (head rows x 64 features, 16 accumulator
  // registers) instead of AMAX x 4 VALU partials per lane
  constexpr bool kMfmaWo = kLateCa;

  // Loads never branch and loaded values are never selected on (which would wait for them):
  // out-of-range positions read a valid address instead -- a sample past m reads sample m - 1
  // (its deltas are zeroed through `valid`), an input column past D reads column D - 1 (it meets a
  // zero W1 column in the forward and lands in a dW1 column the epilogue drops).
  auto fetch = [&](int k) {
    Fetch f;
    const int g0 = (first + k * stride) * 16;
    const int sn = g0 + r;
    f.sn = idxp[sn < mm ? sn : mm - 1];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int st = g0 + 4 * q + v;
      f.st[v] = kLateXt ? 0 : idxp[st < mm ? st : mm - 1];
    }
    return f;
  };
  // a group's layer-1 inputs (N layout) ...
#ifdef DPPO_GATHER_NT  // (A/B) the record gathers with the non-temporal cache policy
#define GLD(p) __builtin_nontemporal_load(p)
#else
#define GLD(p) (*(p))
#endif
  auto gather_xn = [&](const Fetch& f, GRec<NIB>& g) {
    const float* rn = a.rec + (int64_t)f.sn * R;
#pragma unroll
    for (int t = 0; t < 4 * NIB; ++t) {
      const int c = 4 * t + q;
      g.xn[t] = GLD(rn + (c < D ? c : D - 1));
    }
  };
  // ... and the rest of its records
  auto gather_rest = [&](const Fetch& f, GRec<NIB>& g) {
    const float* rn = a.rec + (int64_t)f.sn * R;
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int c = 16 * ib + r;
        g.xt[ib][v] = kLateXt ? 0.f : GLD(a.rec + (int64_t)f.st[v] * R + (c < D ? c : D - 1));
      }
    g.sc = GLD((const f32x4*)(rn + a.D8));
    g.ca[0] = CONT && !kLateCa ? GLD((const f32x4*)(rn + a.D8 + 4)) : z4();
    g.ca[1] = (CONT && !kLateCa && AMAX > 4) ? GLD((const f32x4*)(rn + a.D8 + 8)) : z4();
    g.sn = f.sn;
  };
  auto gather = [&](const Fetch& f) {
    GRec<NIB> g;
    gather_xn(f, g);
    gather_rest(f, g);
    return g;
  };

  // the first groups' indices go out before the weight staging (their gathers wait on them)
  Fetch f_cur{}, f_nxt{};
  if (nk > 0) f_cur = fetch(0);
  if (nk > 1) f_nxt = fetch(1);

  // ---------------- prologue: weights into LDS -- every load is issued before the first store (a
  // load-store loop waits one memory round trip per iteration)
  constexpr int kWLd = 3 * (kMat / 4) / kThreadsW;           // 12 f32x4 of W2 | Wa | Wc per thread
  // W1 image: element k = ((row * 4 + q) * 4 NIB + t) holds W1[row][4t + q], so that lane (q, r)
  // reads the A operands of all its layer-1 k-steps for output block ob as NIB ds_read_b128 at
  // ((16 ob + r) * 4 + q) * 4 NIB (read one float at a time, every k-step's read was waited for
  // right before its MFMA: 4-20 exposed LDS round trips per group)
  constexpr int kW1N = H * 16 * NIB;
  constexpr int kW1Ld = (kW1N + kThreadsW - 1) / kThreadsW;
  static_assert(kW1N <= H * L.RS1, "W1 image");
  static_assert(3 * (kMat / 4) % kThreadsW == 0 && 4 * H == kThreadsW, "prologue split");
  f32x4 wld[kWLd];
  float w1ld[kW1Ld];
#pragma unroll
  for (int i = 0; i < kWLd; ++i) {
    const int k = tid + i * kThreadsW;
    const int mi = k >> 10, e = k & 1023, row = e >> 4, g = e & 15;
    const int64_t off = mi == 0 ? po.W2 : (mi == 1 ? po.Wa : po.Wc);
#ifdef DPPO_ABL_NOSTAGE
    // timing-only ablation (wrong results): no weight loads in the prologue -- the upper bound of
    // what a prebuilt LDS image would save
    wld[i] = (f32x4){(float)off, 0.f, 0.f, (float)(row + g)};
#else
    wld[i] = *(const f32x4*)(P + off + row * H + 4 * g);
#endif
  }
#pragma unroll
  for (int i = 0; i < kW1Ld; ++i) {
    const int k = tid + i * kThreadsW;
    const int t = k % (4 * NIB), qq = (k / (4 * NIB)) & 3, row = k / (16 * NIB), c = 4 * t + qq;
    const bool on = k < kW1N && c < D;
#ifdef DPPO_ABL_NOSTAGE
    w1ld[i] = (float)(on ? row * D + c : 0);
#else
    w1ld[i] = P[po.W1 + (on ? row * D + c : 0)];
#endif
  }
  const float wold = P[po.Wo + ((tid >> 6) < a.A ? tid : 0)];
  const float wold2 = P[po.Wo + ((tid >> 6) + 4 < a.A ? tid + 4 * H : 0)];
  // the small parameters with the weights (loaded where they are stored, behind the weight
  // stores, they cost one more memory round trip before the barrier): Wv, b1, b2, ba, bc of
  // feature tid (tid < H); bo, log std of head h = tid - H and bv (H <= tid < H + 8); every log
  // std for the entropy sums (continuous)
  // (not in the 4-discrete-action instantiation, which has no registers to spare: its main loop
  // would spill)
  constexpr bool kTight = AMAX == 4 && !CONT && NIB == 1;
  constexpr bool kAgprW = !CONT;  // weight-gradient MFMAs in AGPR form (mfma4_acc)
  const int fs = tid < H ? tid : 0;
  const int hs = (tid >= H && tid - H < a.A) ? tid - H : 0;
  float sWv = 0.f, sb1 = 0.f, sb2 = 0.f, sba = 0.f, sbc = 0.f, sbo = 0.f, sls = 0.f, sbv = 0.f;
  float lsv[8];
  if (!kTight) {
    sWv = P[po.Wv + fs];
    sb1 = P[po.b1 + fs];
    sb2 = P[po.b2 + fs];
    sba = P[po.ba + fs];
    sbc = P[po.bc + fs];
    sbo = P[po.bo + hs];
    sls = CONT ? P[po.ls + hs] : 0.0f;
    sbv = P[po.bv];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) lsv[k] = CONT ? P[po.ls + (k < a.A ? k : 0)] : 0.0f;
  GRec<NIB> g_cur{};
  if (nk > 0) g_cur = gather(f_cur);
#pragma unroll
  for (int i = 0; i < kWLd; ++i) {
    const int k = tid + i * kThreadsW;
    const int mi = k >> 10, e = k & 1023, row = e >> 4, g = e & 15;
    *(f32x4*)(lds + L.W2 + mi * H * kWS + row * kWS + 4 * g) = wld[i] * kTS;
  }
#pragma unroll
  for (int i = 0; i < kW1Ld; ++i) {
    const int k = tid + i * kThreadsW;
    const int t = k % (4 * NIB), c = 4 * t + ((k / (4 * NIB)) & 3);
    if (k < kW1N) lds[L.W1 + k] = c < D ? w1ld[i] * kTS : 0.0f;
  }
  lds[L.Wo + tid] = (tid >> 6) < a.A ? wold : 0.0f;
  lds[L.Wo + 4 * H + tid] = (tid >> 6) + 4 < a.A ? wold2 : 0.0f;
  if (tid < H) {
    lds[L.Wv + tid] = kTight ? P[po.Wv + tid] : sWv;
    lds[L.b1 + tid] = (kTight ? P[po.b1 + tid] : sb1) * kTS;
    lds[L.b2 + tid] = (kTight ? P[po.b2 + tid] : sb2) * kTS;
    lds[L.ba + tid] = (kTight ? P[po.ba + tid] : sba) * kTS;
    lds[L.bc + tid] = (kTight ? P[po.bc + tid] : sbc) * kTS;
  } else if (tid < H + 8) {
    const int h = tid - H;
    lds[L.bo + h] = h < a.A ? (kTight ? P[po.bo + h] : sbo) : 0.0f;
    lds[L.ls + h] = (CONT && h < a.A) ? (kTight ? P[po.ls + h] : sls) : 0.0f;
    if (h < 4) lds[L.bv + h] = h == 0 ? (kTight ? P[po.bv] : sbv) : 0.0f;
    if (CONT) {
      // Normal(mean, exp(log_std)) constants of action h (continuous_ppo.py:41-47; torch
      // Normal.log_prob / entropy), the same for every sample
      const bool on = h < a.A;
      const float sg = on ? __expf(kTight ? P[po.ls + h] : sls) : 1.0f;
      lds[L.gc + h] = on ? 1.0f / (2.0f * (sg * sg)) : 0.0f;
      lds[L.gc + 8 + h] = 1.0f / (sg * sg);
      lds[L.gc + 16 + h] = 1.0f / sg;
      lds[L.gc + 24 + h] = on ? __logf(sg) : 0.0f;
      if (h == 0) {
        // (the log-std values were loaded above: a run-time bounded loop here issued the loads
        // one round trip at a time)
        float e = 0.0f, c = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < a.A) {
            const float l = __logf(__expf(lsv[k]));
            e += kHalfLog2PiPlusHalfW + l;  // entropy (continuous_ppo.py:45-47)
            c += l + kLogSqrt2PiW;           // log-prob constant part
          }
        }
        lds[L.gent] = e;
        lds[L.gent + 1] = c;
      }
    }
  }
  __syncthreads();

  const float* W2 = lds + L.W2;
  const float* Wa = W2 + H * kWS;
  const float* Wc = W2 + 2 * H * kWS;
  // the wave's scratch: four [16 x 72] turn slots and the per-sample head-delta image [16][8]
  float* sh1 = lds + L.scratch + wave * kScratch;  // h1 (N -> P), read back for dW2 / dz1
  float* sh2 = sh1 + kSlot;                         // h2 (N -> P), read back for dWa, dWc / dz2
  float* sx = sh2 + kSlot;                          // a1 (N -> P), then dza, then dz2 (P -> N)
  float* sy = sx + kSlot;                           // c1 (N -> P), then dzc
  float* sd = sy + kSlot;                           // {dlogit[0..3], dvalue} per sample

  constexpr int NB1 = X1 ? 1 : NIB;  // input blocks of dW1 on MFMA tiles
  f32x4 gW2[16], gWa[16], gWc[16], gW1[4 * NB1];
#pragma unroll
  for (int i = 0; i < 16; ++i) gW2[i] = gWa[i] = gWc[i] = z4();
#pragma unroll
  for (int i = 0; i < 4 * NB1; ++i) gW1[i] = z4();
  f32x4 gx1 = z4();  // X1: dW1[4r + b][16] partial over this lane's samples 4q + v
  // P-form partials (component b = feature 4r + b, summed over this lane's samples 4q + v)
  f32x4 gb1 = z4(), gb2 = z4(), gba = z4(), gbc = z4(), gWv = z4();
  // gWo[4c + cb][i] = dWo[head 4c + i][feature 4r + cb], partial over this lane's samples
  constexpr int kNWo = kMfmaWo ? 1 : 4 * ((AMAX + 3) / 4);
  f32x4 gWo[kNWo];
#pragma unroll
  for (int h = 0; h < kNWo; ++h) gWo[h] = z4();
  // kMfmaWo: tile cb, lane (q, r), register i = dWo[head 4q + i][feature 4r + cb]
  f32x4 gWoT[4] = {z4(), z4(), z4(), z4()};
  float gbo[AMAX], gls[AMAX], gbv = 0.f, s_pi = 0.f, s_v = 0.f, s_ent = 0.f;
#pragma unroll
  for (int h = 0; h < AMAX; ++h) gbo[h] = gls[h] = 0.f;
#ifdef DPPO_PHASE_TRACE
  WEDGE(1, (long long)__builtin_amdgcn_s_memtime());
#endif

  // ---- (1) layer 1: h1 = tanh(W1 x + b1); k-step t covers inputs {4t + q}.  Group k + 1's runs
  // inside group k's last phase (its 4 MFMAs and tanh beside that phase's 80 weight-gradient
  // MFMAs, instead of a latency-bound phase of its own), so h1 is carried across iterations.
  auto layer1 = [&](f32x4 (&h)[4], const GRec<NIB>& g) {
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) h[ob] = *(const f32x4*)(lds + L.b1 + 16 * ob + 4 * q);
    f32x4 w1[4][NIB];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int tb = 0; tb < NIB; ++tb)
        w1[ob][tb] = *(const f32x4*)(lds + L.W1 + ((16 * ob + r) * 4 + q) * 4 * NIB + 4 * tb);
    // (X1: exactly 17 inputs, 5 k-steps known at compile time -- no run-time branch between the
    // k-steps, so their MFMAs and LDS waits interleave)
    const int nkn = X1 ? 5 : a.nkn;
#pragma unroll
    for (int t = 0; t < 4 * NIB; ++t) {
      if (t < nkn) {
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) h[ob] = mfma4(w1[ob][t >> 2][t & 3], g.xn[t], h[ob]);
      }
    }
    tanh4(h);
    put_n(sh1, h, q, r);
  };
  // (only where the registers allow it: the other instantiations would spill)
  constexpr bool kHoistL1 = !CONT && NIB == 1 && AMAX <= 4;
#ifdef DPPO_MBW_LATE_XN
  constexpr bool kEarlyXn = false;
#else
  constexpr bool kEarlyXn = kHoistL1;
#endif
  f32x4 h1[4];
  if (kHoistL1 && nk > 0) layer1(h1, g_cur);
  PHASE_FENCE();

  for (int k = 0; k < nk; ++k) {
    const int g0 = (first + k * stride) * 16;
    const bool valid = g0 + r < mm;
    WSTAMP(k, 0);
    if (!kHoistL1) {
      layer1(h1, g_cur);
      PHASE_FENCE();
    }
    WSTAMP(k, 1);
    // ---- (2) layer 2
    f32x4 h2[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) h2[ob] = *(const f32x4*)(lds + L.b2 + 16 * ob + 4 * q);
    fwd64(h2, W2, h1, q, r);
    tanh4(h2);
    put_n(sh2, h2, q, r);
    PHASE_FENCE();
    WSTAMP(k, 2);
    // ---- (3) actor / critic hidden layers
    // the actor layer first; the critic layer's MFMAs then run beside the actor's tanh, its
    // scratch turn and the actor head (VALU)
    f32x4 a1[4], c1[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) a1[ob] = *(const f32x4*)(lds + L.ba + 16 * ob + 4 * q);
    fwd64(a1, Wa, h2, q, r);
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) c1[ob] = *(const f32x4*)(lds + L.bc + 16 * ob + 4 * q);
    float out[AMAX];
    if (kLateCa) {
      const float* rn = a.rec + (int64_t)g_cur.sn * R + a.D8;
      g_cur.ca[0] = GLD((const f32x4*)(rn + 4));
      g_cur.ca[1] = GLD((const f32x4*)(rn + 8));
    }
    // the head rows this lane dots (actor heads and the value head), read before the critic
    // layer's MFMAs: read at their use, every row cost one exposed LDS round trip (the scheduler
    // placed each read right before its dot product, after the last MFMA)
    constexpr bool kPreHeads = kPreloadHeads<AMAX, CONT, NIB>();
    // 5-8 heads: the heads are one MFMA output tile instead (A = head row r & 7, the lane's
    // features 16 kb + 4q .. + 3 as for a hidden layer; B = a1): 16 MFMAs against AMAX x 16 VALU
    // FMAs + 4 LDS round trips per head
    constexpr bool kMfmaHeads = AMAX > 4;
    f32x4 wo[kPreHeads ? AMAX : 1][4], wv[4], woT[4];
    if (kMfmaHeads) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) woT[kb] = *(const f32x4*)(lds + L.Wo + (r & 7) * H + 16 * kb + 4 * q);
    }
    if (kPreHeads) {
#pragma unroll
      for (int h = 0; h < AMAX; ++h)
#pragma unroll
        for (int ob = 0; ob < 4; ++ob)
          wo[h][ob] = *(const f32x4*)(lds + L.Wo + h * H + 16 * ob + 4 * q);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) wv[ob] = *(const f32x4*)(lds + L.Wv + 16 * ob + 4 * q);
    }
    SG_FENCE();
    {
      // (reading the critic's first weight block and biases ahead of the head rows, fenced,
      // measured slower at C3: 96.97-97.38 vs 96.24-96.52 us, tools/gpu/r04_w0c.sh)
      fwd64_raw(c1, Wc, h2, q, r);
      tanh4(a1);
      put_n(sx, a1, q, r);
      // ---- (4) heads: logits / means and value of sample r, in every lane of the sample
      if (kPreHeads && !kMfmaHeads) {
        // every head's dot product at once, step by step: AMAX x 2 independent packed chains
        // (pk_dot16's order per head), so that no step waits for its predecessor
        f32x2 pa[kPreHeads ? AMAX : 1], pb[kPreHeads ? AMAX : 1];
#pragma unroll
        for (int h = 0; h < (kPreHeads ? AMAX : 0); ++h) {
          pa[h] = pk_mul(lo2(wo[h][0]), lo2(a1[0]));
          pb[h] = pk_mul(hi2(wo[h][0]), hi2(a1[0]));
        }
#pragma unroll
        for (int ob = 1; ob < 4; ++ob)
#pragma unroll
          for (int h = 0; h < (kPreHeads ? AMAX : 0); ++h) {
            pa[h] = pk_fma(lo2(wo[h][ob]), lo2(a1[ob]), pa[h]);
            pb[h] = pk_fma(hi2(wo[h][ob]), hi2(a1[ob]), pb[h]);
          }
#pragma unroll
        for (int h = 0; h < (kPreHeads ? AMAX : 0); ++h) {
          const f32x2 p = pa[h] + pb[h];
          out[h] = qsum(p[0] + p[1]) + lds[L.bo + h];
        }
      } else {
#pragma unroll
        for (int h = 0; h < (kMfmaHeads ? 0 : AMAX); ++h) {
          float s = 0.f;
#pragma unroll
          for (int ob = 0; ob < 4; ++ob)
            s += dot4(*(const f32x4*)(lds + L.Wo + h * H + 16 * ob + 4 * q), a1[ob]);
          out[h] = qsum(s) + lds[L.bo + h];
        }
      }
      SG_DSR(4 + 4 * AMAX);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (kb < 3) SG_DSR(1);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            SG_MFMA(1);
            SG_VALU(2);
          }
        }
      SG_FENCE();
    }
    if (kMfmaHeads) {
      // two accumulation chains (even / odd k-steps), then tile register v of lane (q, r) = head
      // 4q + v of sample r: rows q = 0 / 1 carry heads 0-3 / 4-7; permlane16_swap gives rows 0-1
      // {row 0, row 1}, permlane32_swap broadcasts the lower half to all four rows
      f32x4 ha = z4(), hb = z4();
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        ha = mfma4(woT[kb][0], a1[kb][0], ha);
        hb = mfma4(woT[kb][1], a1[kb][1], hb);
        ha = mfma4(woT[kb][2], a1[kb][2], ha);
        hb = mfma4(woT[kb][3], a1[kb][3], hb);
      }
      const f32x4 ht = ha + hb;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(ht[v]),
                                                        __float_as_uint(ht[v]), false, false);
        const auto lo = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);
        out[v] = __uint_as_float(lo[0]) + lds[L.bo + v];
        if (4 + v < AMAX) {
          const auto hi = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);
          out[4 + v] = __uint_as_float(hi[0]) + lds[L.bo + 4 + v];
        }
      }
    }
    tanh4(c1);
    put_n(sy, c1, q, r);
    PHASE_FENCE();
    WSTAMP(k, 3);
    // the next group's layer-1 inputs, two phases before the rest of its records: its layer 1
    // runs in this group's phase 9 (kHoistL1), and from phase 7 the records did not always land
    // in time (a 1M-sample record buffer: ~0.8 K cycles per group waited in phase 9 at C3)
    GRec<NIB> g_nxt{};
    if (kEarlyXn && k + 1 < nk) gather_xn(f_nxt, g_nxt);
    // the actor / critic hidden layers in the P layout for the head weight gradients of phase 6,
    // requested now: they land during the loss chain instead of starting phase 6 with a wait
    // (as loaded quads: a1x[v][cb] = feature 4r + cb of sample 4q + v)
    f32x4 a1x[4], c1x[4];
    get_p_raw(a1x, sx, q, r);
    get_p_raw(c1x, sy, q, r);
    // Gaussian heads: the loss phase's constants (1 / (2 var), 1 / var, 1 / sigma per action; the
    // entropy and log-prob-constant sums) as ONE batch of LDS reads here -- read at their use,
    // each was an exposed LDS round trip inside the dependent loss chain (~10 per group)
    constexpr int NG4 = CONT ? (AMAX + 3) / 4 : 1;
    f32x4 kg[3][NG4], kent = z4();
    if (CONT) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int c = 0; c < NG4; ++c) kg[i][c] = *(const f32x4*)(lds + L.gc + 8 * i + 4 * c);
      kent = *(const f32x4*)(lds + L.gent);
    }
    auto kgc = [&](int i, int h) { return CONT ? kg[i][h >> 2][h & 3] : 0.f; };
    // the value head's rows and bias in the same batch (without kPreHeads they were read one
    // row at a time, each waited for right before its dot product)
    f32x4 wvb[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
      wvb[ob] = kPreHeads ? wv[ob] : *(const f32x4*)(lds + L.Wv + 16 * ob + 4 * q);
    const float kbv = lds[L.bv];
    const float vpart = pk_dot16(wvb, c1);
    const float val = qsum(vpart) + kbv;
    // ---- (5) per-sample loss and head deltas (ppo.py:264-280)
    const f32x4 sc = g_cur.sc;
    const float adv = sc[2], ret = sc[3];
    float logp = 0.f, ent = 0.f;
    float p[AMAX], lp[AMAX];
    if (CONT) {
      float qq = 0.f;
#pragma unroll
      for (int h = 0; h < AMAX; ++h) {
        const float d = g_cur.ca[h >> 2][h & 3] - out[h];
        qq += (d * d) * kgc(0, h);  // 1 / (2 var): 0 past A
      }
      logp = -qq - kent[1];
      ent = kent[0];
    } else {
      const int actn = __float_as_int(sc[0]);
      float mx = out[0];
#pragma unroll
      for (int h = 1; h < AMAX; ++h)
        if (h < a.A) mx = fmaxf(mx, out[h]);
      float se = 0.f;
#pragma unroll
      for (int h = 0; h < AMAX; ++h)
        if (h < a.A) se += __expf(out[h] - mx);
      // se >= 1 (its largest term is exp(0)): the bare v_log_f32 (log2) needs no range fix-up
      const float lse = mx + __builtin_amdgcn_logf(se) * kLn2W;
#pragma unroll
      for (int h = 0; h < AMAX; ++h) {
        lp[h] = out[h] - lse;
        p[h] = h < a.A ? __expf(lp[h]) : 0.f;
        ent -= p[h] * lp[h];
        logp = h == actn ? lp[h] : logp;
      }
    }
    const float ratio = __expf(logp - sc[1]);                      // ppo.py:266
    const float rcl = fminf(fmaxf(ratio, 1.0f - a.clip_eps), 1.0f + a.clip_eps);
    const float u = -adv * ratio, w = -adv * rcl;                  // ppo.py:267-269
    const float inr = (ratio >= 1.0f - a.clip_eps && ratio <= 1.0f + a.clip_eps) ? 1.f : 0.f;
    const float gu = u > w ? 1.f : (u == w ? 0.5f : 0.f);          // torch.max splits ties
    const float gw = w > u ? 1.f : (u == w ? 0.5f : 0.f);
    const float vm = valid ? a.inv_m : 0.f;
    const float dlogp = (gu * -adv + gw * -adv * inr) * vm * ratio;
    const float dv = a.vf * (val - ret) * vm;                       // ppo.py:272
    constexpr int NDL = AMAX > 4 ? 8 : 4;
    constexpr int kDv = NDL;  // the value delta follows the logit deltas in a head-delta row
    float dl[NDL];
#pragma unroll
    for (int h = 0; h < NDL; ++h) dl[h] = 0.f;
#pragma unroll
    for (int h = 0; h < AMAX; ++h) {
      if (CONT) {
        const float dd = g_cur.ca[h >> 2][h & 3] - out[h];
        const float zz = dd * kgc(2, h);
        dl[h] = h < a.A ? dlogp * dd * kgc(1, h) : 0.f;
        if (q == 0 && h < a.A) gls[h] += dlogp * (zz * zz - 1.0f);
      } else {
        const int actn = __float_as_int(sc[0]);
        dl[h] = dlogp * ((h == actn ? 1.f : 0.f) - p[h]) + a.ent * vm * p[h] * (lp[h] + ent);
      }
    }
    if (q == 0) {
      if (valid) {
        s_pi += fmaxf(u, w);
        s_v += 0.5f * (val - ret) * (val - ret);
        s_ent += ent;
      }
#pragma unroll
      for (int h = 0; h < AMAX; ++h) gbo[h] += dl[h];
      gbv += dv;
#pragma unroll
      for (int c = 0; c < NDL / 4; ++c)
        *(f32x4*)(sd + kSdw * r + 4 * c) = (f32x4){dl[4 * c], dl[4 * c + 1], dl[4 * c + 2], dl[4 * c + 3]};
      sd[kSdw * r + kDv] = dv;
    }
    PHASE_FENCE();
    WSTAMP(k, 4);
    // kLateXt: the indices of the T-layout input, a phase before its record loads (requested in
    // phase 7 itself, the index -> record chain held the in-order wave for a memory round trip
    // there: 2.2 K cycles of the HalfCheetah group's dh2 phase)
    int st[4];
    if (kLateXt) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int j = g0 + 4 * q + v;
        st[v] = idxp[j < mm ? j : mm - 1];
      }
    }
    // ---- (6) head weight gradients (P layout: feature 4r + cb, samples 4q + v), then the head
    // back-propagation dza = (Wo^T dl)(1 - a1^2), dzc = Wv dv (1 - c1^2) in the N layout
    constexpr bool kPreDh2 = !kTight;  // (it would spill 6 registers there)
    f32x4 dh2_pre[2];
    if (kPreDh2) {
      dh2_pre[0] = bwdP_row(Wa, 0, q, r);
      dh2_pre[1] = bwdP_row(Wa, 1, q, r);
    }
    // 5-8 heads: every LDS operand of this phase as one batch at its start -- the head deltas
    // of the lane's four samples, the head rows of Wo^T dl, the value-head rows -- then a
    // scheduling fence so that none of them sinks to its use (read there, each was an exposed LDS
    // round trip in front of its MFMA: 12 per group)
    float drv[4], dvv[4], woA[2][4];
    f32x4 wvc[4];
    if (kMfmaHeads) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        drv[v] = sd[kSdw * (4 * q + v) + (r < AMAX ? r : 0)];
        dvv[v] = sd[kSdw * (4 * q + v) + kDv];
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) woA[ks][ob] = lds[L.Wo + (4 * ks + q) * H + 16 * ob + r];
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
        wvc[ob] = kPreHeads ? wv[ob] : *(const f32x4*)(lds + L.Wv + 16 * ob + 4 * q);
      SG_FENCE();
    }
    {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if (kMfmaWo) {
          // A operand: the delta of head r of sample 4q + v (rows past the heads are zero)
          const float dr = (kMfmaHeads ? drv[v]
                                       : sd[kSdw * (4 * q + v) + (r < AMAX ? r : 0)]) *
                           (r < AMAX ? 1.f : 0.f);
          const float dvs = kMfmaHeads ? dvv[v] : sd[kSdw * (4 * q + v) + kDv];
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            gWoT[cb] = mfma4(dr, a1x[v][cb], gWoT[cb]);
            gWv[cb] += dvs * c1x[v][cb];
          }
          continue;
        }
        f32x4 d4[NDL / 4];
#pragma unroll
        for (int c = 0; c < NDL / 4; ++c) d4[c] = *(const f32x4*)(sd + kSdw * (4 * q + v) + 4 * c);
        // the value delta with its neighbour as an aligned pair (element 0 broadcast below)
        const f32x2 dvp = *(const f32x2*)(sd + kSdw * (4 * q + v) + kDv);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          // gWo[4c + cb] = dWo partials of heads 4c .. 4c + 3 for feature 4r + cb: the lane's
          // head deltas times a1 (feature 4r + cb, sample 4q + v) broadcast, two packed FMAs
          const f32x2 ap = (cb & 2) ? hi2(a1x[v]) : lo2(a1x[v]);
#pragma unroll
          for (int c = 0; c < (AMAX + 3) / 4; ++c) {
            f32x4& g = gWo[4 * c + cb];
            if (cb & 1)
              g = cat2(pk_fma_bc<1>(lo2(d4[c]), ap, lo2(g)), pk_fma_bc<1>(hi2(d4[c]), ap, hi2(g)));
            else
              g = cat2(pk_fma_bc<0>(lo2(d4[c]), ap, lo2(g)), pk_fma_bc<0>(hi2(d4[c]), ap, hi2(g)));
          }
        }
        // gWv (component cb) += dv * c1 (features 4r + 0..3 of sample 4q + v)
        gWv = cat2(pk_fma_bc<0>(lo2(c1x[v]), dvp, lo2(gWv)), pk_fma_bc<0>(hi2(c1x[v]), dvp, hi2(gWv)));
      }
    }
    f32x4 dza[4], dzc[4];
    // 5-8 heads: Wo^T dl on MFMA (k = head, two k-steps; A = Wo[4ks + q][16 ob + r], B = the
    // delta of head 4ks + q of sample r), the N layout directly
    f32x2 dlp[(AMAX + 1) / 2];
#pragma unroll
    for (int c = 0; c < (AMAX + 1) / 2; ++c) dlp[c] = (f32x2){dl[2 * c], dl[2 * c + 1]};
    float bsel[2];
#pragma unroll
    for (int ks = 0; ks < (kMfmaHeads ? 2 : 0); ++ks)
      bsel[ks] = q == 0 ? dl[4 * ks] : (q == 1 ? dl[4 * ks + 1] : (q == 2 ? dl[4 * ks + 2] : dl[4 * ks + 3]));
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) {
      f32x4 da = z4();
      if (kMfmaHeads) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) da = mfma4(woA[ks][ob], bsel[ks], da);
      } else if (kPreHeads) {
        // sum_h Wo[h] dl[h]: dl[h] broadcast from its pair, two packed FMAs per head (the same
        // operations in the same order as the scalar chain)
        f32x2 alo = pk_mul_bc<0>(lo2(wo[0][ob]), dlp[0]), ahi = pk_mul_bc<0>(hi2(wo[0][ob]), dlp[0]);
#pragma unroll
        for (int h = 1; h < AMAX; ++h) {
          const f32x4 w = wo[kPreHeads ? h : 0][ob];
          if (h & 1) {
            alo = pk_fma_bc<1>(lo2(w), dlp[h >> 1], alo);
            ahi = pk_fma_bc<1>(hi2(w), dlp[h >> 1], ahi);
          } else {
            alo = pk_fma_bc<0>(lo2(w), dlp[h >> 1], alo);
            ahi = pk_fma_bc<0>(hi2(w), dlp[h >> 1], ahi);
          }
        }
        da = cat2(alo, ahi);
      } else {
#pragma unroll
        for (int h = 0; h < AMAX; ++h)
          da += *(const f32x4*)(lds + L.Wo + h * H + 16 * ob + 4 * q) * dl[h];
      }
      dza[ob] = dtanh4(da, a1[ob]);
      dzc[ob] = dtanh4((kMfmaHeads ? wvc[ob]
                                   : (kPreHeads ? wv[ob] : *(const f32x4*)(lds + L.Wv + 16 * ob + 4 * q))) *
                           dv,
                       c1[ob]);
    }
    put_n(sx, dza, q, r);
    put_n(sy, dzc, q, r);
    PHASE_FENCE();
    WSTAMP(k, 5);
    // ---- (7) dh2 = Wa^T dza + Wc^T dzc (P layout)
    if (kLateXt) {
#pragma unroll
      for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int c = 16 * ib + r;
          g_cur.xt[ib][v] = GLD(a.rec + (int64_t)st[v] * R + (c < D ? c : D - 1));
        }
    }
    f32x4 dh2[4] = {z4(), z4(), z4(), z4()};
    if (!kPreDh2) {
      dh2_pre[0] = bwdP_row(Wa, 0, q, r);
      dh2_pre[1] = bwdP_row(Wa, 1, q, r);
    }
    bwdP2(dh2, Wa, dza, Wc, dzc, q, r, dh2_pre);
    // the next group's records (its indices came one group ago) and the indices after that
    if (k + 1 < nk) {
      if (!kEarlyXn) gather_xn(f_nxt, g_nxt);
      gather_rest(f_nxt, g_nxt);
    }
    if (k + 2 < nk) f_nxt = fetch(k + 2);
    PHASE_FENCE();
    WSTAMP(k, 6);
    // ---- (8) dz2 = dh2 (1 - h2^2); hidden-bias partials; dWa, dWc
    {
      f32x4 h2t[4], dzat[4], dzct[4], dz2t[4];
      // h2t first: dz2t needs only it, so its VALU runs while dzat / dzct land
      get_p(h2t, sh2, q, r);
      get_p(dzat, sx, q, r);
      get_p(dzct, sy, q, r);
      // (discrete heads) 1 - h2^2 on the loaded quads (packed), then the transposed product with
      // dh2; the hidden-bias partials of the actor / critic layers, component b, as packed quad
      // sums: (s0 + s1) + (s2 + s3) per component as in the scalar form.  (Gaussian heads keep the
      // scalar form: packed, the X1 kernel measured 0.5 us slower per launch.)
      if constexpr (!CONT) {
        f32x4 g2[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const f32x4 hq = quad_of(h2t, v);
          g2[v] = cat2(pk_fma(-lo2(hq), lo2(hq), (f32x2)(1.0f)), pk_fma(-hi2(hq), hi2(hq), (f32x2)(1.0f)));
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int v = 0; v < 4; ++v) dz2t[b][v] = dh2[b][v] * g2[v][b];
          gb2[b] += (dz2t[b][0] + dz2t[b][1]) + (dz2t[b][2] + dz2t[b][3]);
        }
        gba += (quad_of(dzat, 0) + quad_of(dzat, 1)) + (quad_of(dzat, 2) + quad_of(dzat, 3));
        gbc += (quad_of(dzct, 0) + quad_of(dzct, 1)) + (quad_of(dzct, 2) + quad_of(dzct, 3));
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int v = 0; v < 4; ++v) dz2t[b][v] = dh2[b][v] * (1.0f - h2t[b][v] * h2t[b][v]);
          gba[b] += (dzat[b][0] + dzat[b][1]) + (dzat[b][2] + dzat[b][3]);
          gbc[b] += (dzct[b][0] + dzct[b][1]) + (dzct[b][2] + dzct[b][3]);
          gb2[b] += (dz2t[b][0] + dz2t[b][1]) + (dz2t[b][2] + dz2t[b][3]);
        }
      }
      put_p(sx, dz2t, q, r);
      wgrad<4, kAgprW>(gWa, dzat, h2t);
      wgrad<4, kAgprW>(gWc, dzct, h2t);
    }
    PHASE_FENCE();
    WSTAMP(k, 7);
    // ---- (9) dh1 = W2^T dz2 ; dz1 = dh1 (1 - h1^2) ; dW2 ; dW1
    {
      f32x4 dz2[4], dz2t[4], h1t[4];
      get_n(dz2, sx, q, r);
      // dz2 again in the P layout (from the same slot) and h1 for dW2, requested before the dh1
      // MFMAs so that they land during them (after them in the 4-discrete-action instantiation,
      // which would spill 2 registers)
      if (!kTight) {
        get_p(dz2t, sx, q, r);
        get_p(h1t, sh1, q, r);
      }
      f32x4 dh1[4] = {z4(), z4(), z4(), z4()};
      bwdP(dh1, W2, dz2, q, r);
      if (kTight) {
        get_p(dz2t, sx, q, r);
        get_p(h1t, sh1, q, r);
      }
      // the next group's layer 1 (sh1 is free once h1t is read: one wave's LDS ops run in order)
      if (kHoistL1 && k + 1 < nk) layer1(h1, g_nxt);
      wgrad<4, kAgprW>(gW2, dz2t, h1t);
      f32x4 dz1t[4];
      f32x4 g1[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const f32x4 hq = quad_of(h1t, v);
        g1[v] = cat2(pk_fma(-lo2(hq), lo2(hq), (f32x2)(1.0f)), pk_fma(-hi2(hq), hi2(hq), (f32x2)(1.0f)));
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
          dz1t[b][v] = CONT ? dh1[b][v] * (1.0f - h1t[b][v] * h1t[b][v]) : dh1[b][v] * g1[v][b];
        gb1[b] += (dz1t[b][0] + dz1t[b][1]) + (dz1t[b][2] + dz1t[b][3]);
      }
      wgrad<NB1, kAgprW>(gW1, dz1t, g_cur.xt);
      if (X1) {
        // g_cur.xt[1][v] = input 16 of sample 4q + v in every lane (columns past 16 clamp to it)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int v = 0; v < 4; ++v) gx1[b] += dz1t[b][v] * g_cur.xt[1][v];
      }
    }
    g_cur = g_nxt;
    PHASE_FENCE();
    WSTAMP(k, 8);
  }
  // the epilogue reads the gradient tiles with v_accvgpr_read: the hazard recognizer does not
  // see the asm MFMAs that wrote them, so their wait states are inserted here
  if (kAgprW) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#ifdef DPPO_PHASE_TRACE
  WEDGE(2, (long long)__builtin_amdgcn_s_memtime());
#endif

  // ---------------- epilogue: the four waves' partials summed in LDS in a fixed order
#ifdef DPPO_ABL_HALF_SLABS
  // timing-only ablation (wrong results): the workgroups b with b & 8 -- the same-XCD partners
  // b - 8 under round-robin dispatch -- skip the epilogue entirely, the best case of handing
  // their partial slab to the partner (no LDS sum, no hand-off, no stores): the upper bound of
  // what a pairwise slab reduction could save in this kernel
  if (blockIdx.x & 8) return;
#endif
  float* slab = a.slabs + (int64_t)blockIdx.x * a.slab_stride;
  float* stg0 = lds;
  float* stg1 = lds + kWavesW * kMat;
  float* small = lds + 2 * kWavesW * kMat;
  constexpr int kSmallW = (small_floats(AMAX) + 3) & ~3;
  // dW tile (ob, ib) of lane (q, r), register v = dW[out 16q + 4v + ob][in]: in = 4r + ib for the
  // hidden matrices (both operands in P layout), 16ib + r for W1 (input features in order)
  auto put_hid = [&](float* stg, const f32x4* acc) {
    float* s = stg + wave * kMat;
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        *(f32x4*)(s + (16 * q + 4 * v + ob) * H + 4 * r) =
            (f32x4){acc[ob * 4 + 0][v], acc[ob * 4 + 1][v], acc[ob * 4 + 2][v], acc[ob * 4 + 3][v]};
  };
  float x1s[4];  // X1: the summed column-16 partials (filled below)
  auto put_w1 = [&](float* stg, const f32x4* acc) {
    float* s = stg + wave * kMat;
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int ib = 0; ib < NB1; ++ib) {
        const int col = 16 * ib + r;
        if (col < D) {
#pragma unroll
          for (int v = 0; v < 4; ++v) s[(16 * q + 4 * v + ob) * D + col] = acc[ob * NB1 + ib][v];
        }
      }
    if (X1 && q == 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) s[(4 * r + b) * D + 16] = x1s[b];
    }
  };
  auto sum_mat = [&](const float* stg, int64_t off, int n4, float scale) {
    for (int c = tid; c < n4; c += kThreadsW) {
      const f32x4 v = ((((const f32x4*)stg)[c] + ((const f32x4*)(stg + kMat))[c]) +
                       ((const f32x4*)(stg + 2 * kMat))[c]) +
                      ((const f32x4*)(stg + 3 * kMat))[c];
      const f32x4 w = scale == 1.0f ? v : v * scale;
      if (a.plain_slab) *(f32x4*)(slab + off + 4 * c) = w;
      else slab_st4(slab + off + 4 * c, w);
    }
  };
  // a whole hidden matrix: all sixteen LDS reads of a thread in flight before the first add
  auto sum_hid = [&](const float* stg, int64_t off, float scale) {
    constexpr int kIt = kMat / 4 / kThreadsW;
    f32x4 x[kIt][4];
#pragma unroll
    for (int i = 0; i < kIt; ++i)
#pragma unroll
      for (int w = 0; w < 4; ++w) x[i][w] = ((const f32x4*)(stg + w * kMat))[tid + i * kThreadsW];
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      const f32x4 v = ((x[i][0] + x[i][1]) + x[i][2]) + x[i][3];
      const f32x4 w = scale == 1.0f ? v : v * scale;
      if (a.plain_slab) *(f32x4*)(slab + off + 4 * (tid + i * kThreadsW)) = w;
      else slab_st4(slab + off + 4 * (tid + i * kThreadsW), w);
    }
  };
  // register-only reductions of this wave's small items first (they overlap the wait for the
  // slowest wave): hidden biases and head weights (P form: sum over q), head biases / log-std /
  // loss sums (every lane: 16-lane rows by DPP, then the four rows)
  float xs[4][5 + AMAX];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    x1s[b] = X1 ? qsum(gx1[b]) : 0.f;
    xs[b][0] = qsum(gb1[b]);
    xs[b][1] = qsum(gb2[b]);
    xs[b][2] = qsum(gba[b]);
    xs[b][3] = qsum(gbc[b]);
    xs[b][4] = qsum(gWv[b]);
#pragma unroll
    for (int h = 0; h < AMAX; ++h) xs[b][5 + h] = kMfmaWo ? 0.f : qsum(gWo[kMfmaWo ? 0 : 4 * (h >> 2) + b][h & 3]);
  }
  float sc[2 * AMAX + 4];
#pragma unroll
  for (int h = 0; h < AMAX; ++h) {
    sc[h] = gbo[h];
    sc[AMAX + h] = gls[h];
  }
  sc[2 * AMAX] = gbv;
  sc[2 * AMAX + 1] = s_pi;
  sc[2 * AMAX + 2] = s_v;
  sc[2 * AMAX + 3] = s_ent;
#pragma unroll
  for (int j = 0; j < 2 * AMAX + 4; ++j) sc[j] = qsum(row16(sc[j]));
  __syncthreads();  // every wave is done with the weights and its scratch
  ESTAMP(0);
  put_hid(stg0, gW2);
  put_hid(stg1, gWa);
  {
    float* s = small + wave * kSmallW;
    if (q == 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int f = 4 * r + b;
        s[0 * H + f] = xs[b][0];
        s[1 * H + f] = xs[b][1];
        s[2 * H + f] = xs[b][2];
        s[3 * H + f] = xs[b][3];
        if (!kMfmaWo) {
#pragma unroll
          for (int h = 0; h < AMAX; ++h) s[4 * H + h * H + f] = xs[b][5 + h];
        }
        s[(4 + AMAX) * H + f] = xs[b][4];
      }
    }
    if (kMfmaWo && 4 * q < AMAX) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (4 * q + i < AMAX) s[4 * H + (4 * q + i) * H + 4 * r + cb] = gWoT[cb][i];
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 2 * AMAX + 4; ++j) s[(5 + AMAX) * H + j] = sc[j];
    }
  }
  ESTAMP(1);
  __syncthreads();
  ESTAMP(2);
  sum_hid(stg0, po.W2, kInvTS);
  sum_hid(stg1, po.Wa, 1.0f);
  for (int j = tid; j < kSmallW; j += kThreadsW) {
    const float v = ((small[j] + small[kSmallW + j]) + small[2 * kSmallW + j]) +
                    small[3 * kSmallW + j];
    if (j < 4 * H) {
      const int l = j >> 6, f = j & 63;
      const int64_t off = l == 0 ? po.b1 : (l == 1 ? po.b2 : (l == 2 ? po.ba : po.bc));
      slab[off + f] = l == 0 ? v * kInvTS2 : (l == 1 ? v * kInvTS : v);
    } else if (j < (4 + AMAX) * H) {
      const int h = (j - 4 * H) >> 6, f = j & 63;
      if (h < a.A) slab[po.Wo + h * H + f] = v;
    } else if (j < (5 + AMAX) * H) {
      slab[po.Wv + (j - (4 + AMAX) * H)] = v;
    } else {
      const int e = j - (5 + AMAX) * H;
      if (e < AMAX) {
        if (e < a.A) slab[po.bo + e] = v;
      } else if (e < 2 * AMAX) {
        if (CONT && e - AMAX < a.A) slab[po.ls + (e - AMAX)] = v;
      } else if (e == 2 * AMAX) {
        slab[po.bv] = v;
      } else if (e < 2 * AMAX + 4) {
        slab[a.p_total + (e - 2 * AMAX - 1)] = v;
      }
    }
  }
  ESTAMP(3);
  __syncthreads();  // stg0 / stg1 reused
  put_hid(stg0, gWc);
  put_w1(stg1, gW1);
  ESTAMP(4);
  __syncthreads();
  ESTAMP(5);
  sum_hid(stg0, po.Wc, 1.0f);
  sum_mat(stg1, po.W1, H * D / 4, kInvTS2);
  ESTAMP(6);
#ifdef DPPO_PHASE_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  WEDGE(3, (long long)__builtin_amdgcn_s_memtime());
  WEDGE(5, (long long)__builtin_amdgcn_s_memrealtime());
#endif
}

}  // namespace

#ifdef DPPO_PHASE_TRACE
extern "C" __attribute__((visibility("default"))) int dppo_debug_mbw_edges(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mbw_edges), sizeof(g_mbw_edges)) == hipSuccess
             ? 0
             : -2;
}
extern "C" __attribute__((visibility("default"))) int dppo_debug_mbw_epi(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mbw_epi), sizeof(g_mbw_epi)) == hipSuccess ? 0 : -2;
}
extern "C" __attribute__((visibility("default"))) int dppo_debug_mbw_phase(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mbw_phase), sizeof(g_mbw_phase)) == hipSuccess
             ? 0
             : -2;
}
#endif

bool mbw_supported(const MlpShape& sh) {
  static const int legacy = [] {
    const char* e = std::getenv("DPPO_MB_LEGACY");
    return e && e[0] == '1' ? 1 : 0;
  }();
  // Up to 4 actions at any input width; 5-8 for discrete heads on <= 16 inputs; 5-6 Gaussian
  // actions on exactly 17 inputs (HalfCheetah: the X1 instantiation, spill-free, 74 vs 77.5 us per
  // launch of the two-team kernel).  The rest goes to the two-team kernel: their sample-split
  // instantiations spill.
  if (legacy || sh.D > 32) return false;
  // DPPO_MBW_CONT6 (A/B): 0 sends the 17-input shape to the two-team kernel too, 1 sends 5-6
  // Gaussian actions on any 17-32 inputs to the sample-split kernel
  static const int cont6 = [] {
    const char* e = std::getenv("DPPO_MBW_CONT6");
    return e && e[0] ? e[0] - '0' : -1;
  }();
  if (sh.continuous && sh.A >= 5 && sh.A <= 6 && sh.D > 16) {
    if (cont6 == 1) return true;
    return cont6 != 0 && sh.D == 17;
  }
  return sh.A <= 4 || (sh.A <= 8 && !sh.continuous && sh.D <= 16);
}

int mbw_grid(int32_t m) {
  int g = (m + 63) / 64;  // 64 samples per workgroup round (4 waves x 16)
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  return g;
}

size_t mbw_lds_bytes(const MlpShape& sh) {
  const int D16 = (sh.D + 15) / 16 * 16;
  const WLds L = make_wlds(D16);
  const int epi = epi_floats(sh.A <= 2 ? 2 : (sh.A <= 4 ? 4 : 8));
  const int n = L.total > epi ? L.total : epi;
  return (size_t)n * sizeof(float);
}

int launch_mbw(const MlpShape& sh, const ParamOffsets& po, const GradArgs& ga, int G,
               hipStream_t s) {
  WArgs k{};
  const int D16 = (sh.D + 15) / 16 * 16;
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
  k.A = sh.A;
  k.R = sh.R;
  k.nkn = (sh.D + 3) / 4;
  static const int plain = [] {
    const char* e = std::getenv("DPPO_SLAB_PLAIN");
    return e && e[0] == '1' ? 1 : 0;
  }();
  k.plain_slab = plain;
  const size_t lds = mbw_lds_bytes(sh);
  if (lds > 160 * 1024) {
    set_error("minibatch kernel needs %zu bytes of LDS (> 160 KiB)", lds);
    return DPPO_EUNSUPPORTED;
  }
  static const bool attr = [] {
#define DPPO_SETW(A, C, N) raise_dyn_lds((const void*)mbw_kernel<A, C, N>);
    DPPO_SETW(2, false, 1) DPPO_SETW(2, true, 1) DPPO_SETW(4, false, 1) DPPO_SETW(4, true, 1)
    DPPO_SETW(2, false, 2) DPPO_SETW(2, true, 2) DPPO_SETW(4, false, 2) DPPO_SETW(4, true, 2)
    DPPO_SETW(8, false, 1) DPPO_SETW(6, true, 2)
#undef DPPO_SETW
    raise_dyn_lds((const void*)mbw_kernel<6, true, 2, true>);
    return true;
  }();
  (void)attr;
  const dim3 grid((unsigned)G), block(kThreadsW);
  const bool c = sh.continuous != 0;
  const bool n2 = D16 > 16;
#define DPPO_LW(A, C, N) DPPO_LAUNCH((mbw_kernel<A, C, N>), grid, block, lds, s, k)
#define DPPO_LWC(A)                      \
  do {                                   \
    if (n2) {                            \
      if (c) DPPO_LW(A, true, 2);        \
      else DPPO_LW(A, false, 2);         \
    } else {                             \
      if (c) DPPO_LW(A, true, 1);        \
      else DPPO_LW(A, false, 1);         \
    }                                    \
  } while (0)
  if (sh.A <= 2) DPPO_LWC(2);
  else if (sh.A <= 4) DPPO_LWC(4);
  else if (c && sh.D == 17) DPPO_LAUNCH((mbw_kernel<6, true, 2, true>), grid, block, lds, s, k);
  else if (c) DPPO_LW(6, true, 2);  // mbw_supported: 5-6 Gaussian actions, 17-32 inputs
  else DPPO_LW(8, false, 1);  // mbw_supported: discrete, D <= 16
#undef DPPO_LWC
#undef DPPO_LW
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
