// Default actor-critic MLP (hidden 64) on gfx950 fp32 MFMA: old-policy evaluation.
//
// Reference: ActorCriticNetwork (diamond/ppo.py:40-96), ContinuousActorCriticNetwork
// (diamond/continuous_ppo.py:50-111), old-policy eval (ppo.py:235-238,
// continuous_ppo.py:247-250).  The fused minibatch kernel is mbstep.hip.
//
// ---- Tiling -----------------------------------------------------------------------------------
// Activations are FEATURE-major: a [64 features x 32 samples] activation is two 32x32 MFMA
// accumulator tiles (f32x16 per lane) of v_mfma_f32_32x32x2_f32, sample on the lane
// (col = lane & 31), features in the 16 registers (row = (r&3) + 8(r>>2) + 4(lane>>5)).
// A layer Y = W X + b then sums over X's ROW index, so X's accumulator registers ARE the next
// MFMA's B operand with no data movement (k-step r uses rows krow(r,0) and krow(r,1) = +4);
// the A operand is the matching W element, read from an LDS image of W (row stride 68 floats:
// conflict-free ds_read_b128 of W[o][k..k+3]).  All math is exact fp32 (f32-input MFMA = an
// ordered fmaf chain, no xf32 on gfx950); tanh is one exp and one hardware reciprocal.
//
// ---- Work decomposition -----------------------------------------------------------------------
// 512-thread workgroups, two per CU (the weight image is ~58 KB of LDS per workgroup), so four
// waves per SIMD interleave their MFMA chains with each other's tanh / head VALU work.  Each wave
// walks 32-sample tiles; the layers are evaluated in an order that keeps at most two activation
// blocks live (h1 -> h2 -> critic -> value -> actor -> heads), under the 128-VGPR budget of four
// waves per SIMD.
#include "common.h"

namespace dppo {
namespace {

constexpr int H = 64;
constexpr int SW = H + 4;  // LDS row stride (floats) of the H-wide weight images
constexpr int kThreads = 512;
constexpr int kWaves = kThreads / kWave;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
// Hidden-layer weights and biases are staged into LDS pre-multiplied by kTS = 2 log2(e): the
// MFMAs then produce kTS z and tanh_inplace skips its multiply (one VALU instruction fewer per
// activation; VALU is not hidden behind fp32 MFMAs on gfx950).
constexpr float kTS = 2.8853900817779268f;
constexpr int kQueueCap = 256;  // a wave's ring of queued critic-pass samples (power of 2, >= 96)
constexpr int kMatchRound = 4;  // next_obs / obs feature pairs compared per round of loads

// LDS image (floats).  Every offset is a compile-time constant, so the weight and bias reads
// take it as an instruction immediate from one base register; only the layer-1 image's row stride
// S1 = D8 + 4 is a run-time value (the image sits last among the weights, sized for D8 <= 32).
// (With run-time offsets the eval kernel held ~15 of them in SGPRs and spilled 45 SGPRs into VGPR
// lanes: v_writelane / v_readlane + hazard s_nops inside the tile loop.)
struct LdsLayout {
  static constexpr int W2 = 0, Wa = H * SW, Wc = 2 * H * SW;  // [H][SW]
  static constexpr int Wo = 3 * H * SW;                      // [A][H]  (logits or mean head)
  static constexpr int kWoCap = 16 * H;                      // up to 16 heads
  static constexpr int Wv = Wo + kWoCap;                     // [H]
  static constexpr int b1 = Wv + H, b2 = b1 + H, ba = b2 + H, bc = ba + H;  // [H]
  static constexpr int bo = bc + H, ls = bo + 32;            // [32]
  static constexpr int bv = ls + 32;                         // [4]
  static constexpr int W1 = bv + 4;                          // [H][S1], zero columns D..S1
  static constexpr int kS1Max = 36;
  static constexpr int weights_end = W1 + H * kS1Max;
  static constexpr int queue = weights_end;  // [kWaves][kQueueCap] int32 (eval_kernel reuse ring)
  static constexpr int total = queue + kWaves * kQueueCap + 2 * kWaves;  // + ring counts / heads
  int S1;
};
static_assert(LdsLayout::W1 % 4 == 0 && LdsLayout::Wo % 4 == 0, "16-B aligned images");

struct KArgs {
  LdsLayout L;
  ParamOffsets po;
  const float* params;
  const float* obs;
  const void* actions;
  const float* next_obs;
  float *logp, *values, *next_values;
  int64_t n;
  // shapes
  int D, D8, nq1, A, R;
  int q4;  // obs (and next_obs) rows of a multiple of 4 floats in 16-B aligned buffers
  // next-value reuse (EvalReuse): row > 0 = the buffers are a [T][row] rollout
  int64_t row;
};

__host__ __device__ inline int align4(int x) { return (x + 3) & ~3; }

LdsLayout make_layout(const MlpShape& sh) {
  LdsLayout L{};
  L.S1 = sh.D8 + 4;
  return L;
}

// ------------------------------------------------------------------------------------------------
// A per-iteration opaque copy of the LDS base.  Weight reads are loop-invariant, and without this
// the compiler hoists every one of them out of the tile loop into ~250 registers (then spills);
// reading them next to their MFMAs costs one ds_read per 1-4 MFMAs instead.
__device__ __forceinline__ float* opaque_base(float* p) {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return p + z;
}

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void load_weights(float* lds, const KArgs& a, int tid) {
  const float* P = a.params;
  const LdsLayout& L = a.L;
  for (int k = tid; k < H * L.S1; k += kThreads) {
    const int o = k / L.S1, c = k % L.S1;
    lds[L.W1 + k] = c < a.D ? P[a.po.W1 + o * a.D + c] * kTS : 0.0f;
  }
  for (int k = tid; k < H * H; k += kThreads) {
    const int o = k >> 6, c = k & 63;
    lds[L.W2 + o * SW + c] = P[a.po.W2 + k] * kTS;
    lds[L.Wa + o * SW + c] = P[a.po.Wa + k] * kTS;
    lds[L.Wc + o * SW + c] = P[a.po.Wc + k] * kTS;
  }
  for (int k = tid; k < a.A * H; k += kThreads) lds[L.Wo + k] = P[a.po.Wo + k];
  for (int k = tid; k < H; k += kThreads) {
    lds[L.Wv + k] = P[a.po.Wv + k];
    lds[L.b1 + k] = P[a.po.b1 + k] * kTS;
    lds[L.b2 + k] = P[a.po.b2 + k] * kTS;
    lds[L.ba + k] = P[a.po.ba + k] * kTS;
    lds[L.bc + k] = P[a.po.bc + k] * kTS;
  }
  for (int k = tid; k < 32; k += kThreads) {
    lds[L.bo + k] = k < a.A ? P[a.po.bo + k] : 0.0f;
    lds[L.ls + k] = (a.po.ls >= 0 && k < a.A) ? P[a.po.ls + k] : 0.0f;
  }
  if (tid < 4) lds[L.bv + tid] = tid == 0 ? P[a.po.bv] : 0.0f;
}

// Bias-initialised accumulator for output block ob: reg r <- b[ob*32 + krow(r, h)].
__device__ __forceinline__ f32x16 bias_block(const float* b, int ob, int h) {
  f32x16 acc;
  const float* bp = b + ob * 32 + 4 * h;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 v = *(const f32x4*)(bp + 8 * q);
    acc[4 * q + 0] = v[0];
    acc[4 * q + 1] = v[1];
    acc[4 * q + 2] = v[2];
    acc[4 * q + 3] = v[3];
  }
  return acc;
}

// Sixteen activations stage by stage from pre-scaled inputs x = kTS z: tanh z = 1 - 2 / (2^x + 1),
// four instructions each (v_exp, v_rcp and two plain ones; saturates through 2^x = inf / 0;
// absolute error <= ~1.2e-7), consecutive instructions independent (mbwave.hip tanh4).
// The two plain steps as packed instructions on the accumulator's register pairs (two elements
// per v_pk_add_f32 / v_pk_fma_f32 at the issue cost of one scalar instruction beside the MFMAs,
// tools/probe/mfma_kind.py).
__device__ __forceinline__ void tanh_inplace(f32x16& x) {
  f32x2 e[8];
#pragma unroll
  for (int r = 0; r < 16; ++r) e[r >> 1][r & 1] = __builtin_amdgcn_exp2f(x[r]);
#pragma unroll
  for (int p = 0; p < 8; ++p) e[p] = e[p] + 1.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) e[r >> 1][r & 1] = __builtin_amdgcn_rcpf(e[r >> 1][r & 1]);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const f32x2 y = __builtin_elementwise_fma((f32x2)(-2.0f), e[p], (f32x2)(1.0f));
    x[2 * p] = y[0];
    x[2 * p + 1] = y[1];
  }
}

// part + part of lane ^ 32 with v_permlane32_swap (a VALU lane move, no LDS round trip); the
// same two operands in both halves
__device__ __forceinline__ float half_sum(float part) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part),
                                                  false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}

// out = tanh(W X + b), W: [64][64] LDS image (stride SW), X: 2 k-blocks.
__device__ __forceinline__ void dense_tanh(f32x16 (&out)[2], const float* W, const float* b,
                                           const f32x16 (&x)[2], int l31, int h) {
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    f32x16 acc = bias_block(b, ob, h);
    const float* wp = W + (ob * 32 + l31) * SW + 4 * h;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 w = *(const f32x4*)(wp + kb * 32 + 8 * q);
        acc = mfma(w[0], x[kb][4 * q + 0], acc);
        acc = mfma(w[1], x[kb][4 * q + 1], acc);
        acc = mfma(w[2], x[kb][4 * q + 2], acc);
        acc = mfma(w[3], x[kb][4 * q + 3], acc);
      }
    }
    tanh_inplace(acc);
    out[ob] = acc;
    __builtin_amdgcn_sched_barrier(0);
  }
}

// First layer: K = D8 (<= 32) features in one k-block, nq1 = D8/8 groups of 4 k-steps.
__device__ __forceinline__ void dense1_tanh(f32x16 (&out)[2], const float* W1, int S1,
                                            const float* b, const f32x16& x0, int nq1, int l31,
                                            int h) {
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    f32x16 acc = bias_block(b, ob, h);
    const float* wp = W1 + (ob * 32 + l31) * S1 + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq1) {
        const f32x4 w = *(const f32x4*)(wp + 8 * q);
        acc = mfma(w[0], x0[4 * q + 0], acc);
        acc = mfma(w[1], x0[4 * q + 1], acc);
        acc = mfma(w[2], x0[4 * q + 2], acc);
        acc = mfma(w[3], x0[4 * q + 3], acc);
      }
    }
    tanh_inplace(acc);
    out[ob] = acc;
  }
}







// Per-sample head: out[a] = Wo[a] . x + bo[a] with x = a 64-feature activation (2 blocks);
// each lane half holds 32 of the features, the two halves are combined with a lane swap.
template <int AMAX>
__device__ __forceinline__ void heads(float (&out)[AMAX], const float* Wo, const float* bo,
                                      int A, const f32x16 (&x)[2], int h) {
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    float part = 0.0f;
    if (a < A) {
      // a 32-feature block's four 16-B slices read together (one at a time, each read was
      // waited for right before its dot product)
      // (16 heads: their instantiation would spill, one read at a time there)
      const float* wp = Wo + a * H + 4 * h;
      // packed pair products (two elements per v_pk_fma_f32) in two independent chains, summed
      // once at the end
      f32x2 pa = (f32x2)(0.0f), pb = (f32x2)(0.0f);
#pragma unroll
      for (int fb = 0; fb < 2; ++fb) {
        f32x4 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (AMAX <= 8) w[q] = *(const f32x4*)(wp + fb * 32 + 8 * q);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 wq = AMAX <= 8 ? w[q] : *(const f32x4*)(wp + fb * 32 + 8 * q);
          pa = __builtin_elementwise_fma((f32x2){wq[0], wq[1]},
                                         (f32x2){x[fb][4 * q + 0], x[fb][4 * q + 1]}, pa);
          pb = __builtin_elementwise_fma((f32x2){wq[2], wq[3]},
                                         (f32x2){x[fb][4 * q + 2], x[fb][4 * q + 3]}, pb);
        }
      }
      const f32x2 pp = pa + pb;
      part = pp[0] + pp[1];
    }
    out[a] = half_sum(part) + bo[a];
  }
}

__device__ __forceinline__ float value_head(const float* Wv, float bv, const f32x16 (&x)[2],
                                            int h) {
  const float* wp = Wv + 4 * h;
  f32x2 pa = (f32x2)(0.0f), pb = (f32x2)(0.0f);
#pragma unroll
  for (int fb = 0; fb < 2; ++fb) {
    f32x4 w[4];  // a block's four slices read together (heads above)
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = *(const f32x4*)(wp + fb * 32 + 8 * q);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pa = __builtin_elementwise_fma((f32x2){w[q][0], w[q][1]},
                                     (f32x2){x[fb][4 * q + 0], x[fb][4 * q + 1]}, pa);
      pb = __builtin_elementwise_fma((f32x2){w[q][2], w[q][3]},
                                     (f32x2){x[fb][4 * q + 2], x[fb][4 * q + 3]}, pb);
    }
  }
  const f32x2 pp = pa + pb;
  return half_sum(pp[0] + pp[1]) + bv;
}



// A lane's layer-1 inputs: x[4q + j] = feature 8q + 4h + j of its sample (zero past D).
// (q4: rows of a multiple of 4 features in 16-B aligned buffers, checked on the host)
__device__ __forceinline__ f32x16 load_x0_obs(const float* o, int D, int nq1, bool valid, int h,
                                              bool q4) {
  // (entries of k-groups q >= nq1 stay unset: dense1_tanh reads only q < nq1 -- zeroing all 16
  // was 16 v_mov per call; an invalid sample's column is never stored)
  f32x16 x;
  if (q4) {
    // rows of a multiple of 4 features (16-B aligned): four features are one 16-B load (four
    // 4-B loads under per-feature exec masks before), no branch: the address is always valid (a
    // block past D reads the row's last one, an invalid sample row 0) and the select drops it
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq1) {
        const int f = 8 * q + 4 * h;
        const f32x4 v = *(const f32x4*)(o + (f < D ? f : D - 4));
        const bool on = valid && f < D;
#pragma unroll
        for (int j = 0; j < 4; ++j) x[4 * q + j] = on ? v[j] : 0.0f;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f = 8 * q + 4 * h + j;
          x[4 * q + j] = (valid && f < D) ? o[f] : 0.0f;
        }
      }
    }
  }
  return x;
}

// ------------------------------------------------------------------------------------------------
// Old-policy evaluation (ppo.py:235-238): one wave per 32-sample tile, grid-stride over tiles.
template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 4) void eval_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  load_weights(lds_, a, tid);
  __syncthreads();
  const LdsLayout& L = a.L;
  const float bv = lds_[L.bv];
  const int64_t ntiles = (a.n + 31) / 32;
  // Reuse mode (a.row > 0, the buffers are a [T][row] rollout): the samples whose next value
  // needs a critic pass on next_obs are queued in a wave-private LDS ring, and the wave runs that
  // pass itself, 32 queued samples at a time (and the remainder at the end) -- no global list, no
  // second kernel, no copy pass.  (Queue head / fill kept wave-uniform -- scalar registers: the
  // vector ones are all taken at four waves per SIMD.)
  const int qbase = L.queue + __builtin_amdgcn_readfirstlane(wave) * kQueueCap;
  int qh = 0, qn = 0;
  // critic pass (get_values, ppo.py:84-89) on next_obs of the first `cnt` queued samples: the
  // same instructions as the obs pass's critic, so a sample's next value has the same bits
  // whichever tile computes it
  // critic pass on sample k of each lane (qv: the lane has one)
  auto critic_tile = [&](bool qv, int64_t k) {
    float* lds = opaque_base(lds_);
    f32x16 x[2], y[2];
    x[0] = load_x0_obs(a.next_obs + k * a.D, a.D, a.nq1, qv, h, a.q4);
    dense1_tanh(y, lds + L.W1, L.S1, lds + L.b1, x[0], a.nq1, l31, h);
    dense_tanh(x, lds + L.W2, lds + L.b2, y, l31, h);
    dense_tanh(y, lds + L.Wc, lds + L.bc, x, l31, h);
    const float nv = value_head(lds + L.Wv, bv, y, h);
    if (qv && h == 0) a.next_values[k] = nv;
  };
  auto critic_queue = [&](int cnt) {
    const bool qv = l31 < cnt;
    const int64_t k = qv ? ((const int32_t*)lds_)[qbase + ((qh + l31) & (kQueueCap - 1))] : 0;
    critic_tile(qv, k);
    qh = (qh + cnt) & (kQueueCap - 1);
    qn -= cnt;
  };
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles;
       tile += (int64_t)gridDim.x * kWaves) {
    float* lds = opaque_base(lds_);
    const int64_t i = tile * 32 + l31;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : 0;
    // the sampled action (categorical), requested with the observation: read at its use after
    // the heads, it was one more memory round trip per tile
    const int act_d = CONT ? 0 : ((const int32_t*)a.actions)[ic];
    // ---- obs: full actor-critic forward (get_logits_and_values, ppo.py:91-96)
    f32x16 x[2], y[2];
    x[0] = load_x0_obs(a.obs + ic * a.D, a.D, a.nq1, valid, h, a.q4);
    dense1_tanh(y, lds + L.W1, L.S1, lds + L.b1, x[0], a.nq1, l31, h);       // y = h1
    dense_tanh(x, lds + L.W2, lds + L.b2, y, l31, h);                         // x = h2
    dense_tanh(y, lds + L.Wc, lds + L.bc, x, l31, h);                         // y = critic hidden
    const float v = value_head(lds + L.Wv, bv, y, h);
    dense_tanh(y, lds + L.Wa, lds + L.ba, x, l31, h);                         // y = actor hidden
    float out[AMAX];
    heads<AMAX>(out, lds + L.Wo, lds + L.bo, a.A, y, h);
    float logp;
    if (CONT) {
      // JointNormal.log_prob (continuous_ppo.py:41-43; torch Normal.log_prob)
      const float* act = (const float*)a.actions + ic * a.A;
      logp = 0.0f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        if (k < a.A) {
          const float ls = lds[L.ls + k];
          const float sc = expf(ls);
          const float d = act[k] - out[k];
          logp += -(d * d) / (2.0f * (sc * sc)) - logf(sc) - kLogSqrt2Pi;
        }
      }
    } else {
      // Categorical(logits).log_prob (torch distributions/categorical.py:78,156)
      const int act = act_d;
      float mx = out[0];
#pragma unroll
      for (int k = 1; k < AMAX; ++k)
        if (k < a.A) mx = fmaxf(mx, out[k]);
      float se = 0.0f, za = out[0];
#pragma unroll
      for (int k = 0; k < AMAX; ++k)
        if (k < a.A) {
          se += expf(out[k] - mx);
          if (k == act) za = out[k];
        }
      logp = za - (mx + logf(se));
    }
    if (a.row > 0) {
      // next_obs[i - row] bitwise equal to this sample's obs[i] (the reference's rollout stores
      // the same array for both unless the env was reset, ppo.py:163-179): V(next_obs[i - row]) is
      // this tile's v, computed by the same instructions on the same bits -- written here.  The
      // other predecessors, and the samples of the last row (no successor), are queued for the
      // wave's critic pass.
      const int64_t ip = i - a.row;
      bool need_p = false, need_s = false;
      if (valid && h == 0) {
        need_s = i + a.row >= a.n;
        if (ip >= 0) {
          bool m = true;
          // kMatchRound features per round, all their loads in flight together (a short-circuit
          // loop waited for every pair: D memory round trips per tile)
          const uint32_t* p = (const uint32_t*)(a.next_obs + ip * a.D);
          const uint32_t* o = (const uint32_t*)(a.obs + ic * a.D);
          if (a.q4) {
            // 16-B rows: kMatchRound 4-feature pairs per round of loads
            for (int f0 = 0; f0 < a.D; f0 += 4 * kMatchRound) {
              u32x4 pv[kMatchRound], ov[kMatchRound];
#pragma unroll
              for (int j = 0; j < kMatchRound; ++j) {
                const int f = f0 + 4 * j < a.D ? f0 + 4 * j : a.D - 4;
                pv[j] = *(const u32x4*)(p + f);
                ov[j] = *(const u32x4*)(o + f);
              }
#pragma unroll
              for (int j = 0; j < kMatchRound; ++j)
                m = m & (pv[j][0] == ov[j][0]) & (pv[j][1] == ov[j][1]) & (pv[j][2] == ov[j][2]) &
                    (pv[j][3] == ov[j][3]);
            }
          } else {
            for (int f0 = 0; f0 < a.D; f0 += kMatchRound) {
              uint32_t pv[kMatchRound], ov[kMatchRound];
#pragma unroll
              for (int j = 0; j < kMatchRound; ++j) {
                const int f = f0 + j < a.D ? f0 + j : a.D - 1;
                pv[j] = p[f];
                ov[j] = o[f];
              }
#pragma unroll
              for (int j = 0; j < kMatchRound; ++j) m = m & (pv[j] == ov[j]);
            }
          }
          if (m) a.next_values[ip] = v;
          need_p = !m;
        }
        a.logp[i] = logp;
        a.values[i] = v;
      }
      // enqueue (ring of kQueueCap; at most 64 per tile onto < 32 left, so it never overflows)
      const uint64_t bp = __ballot(need_p), bs = __ballot(need_s);
      const uint64_t below = (1ull << lane) - 1ull;
      int32_t* qr = (int32_t*)lds_ + qbase;
      if (need_p) qr[(qh + qn + __popcll(bp & below)) & (kQueueCap - 1)] = (int32_t)ip;
      const int np = __builtin_amdgcn_readfirstlane(__popcll(bp));
      if (need_s) qr[(qh + qn + np + __popcll(bs & below)) & (kQueueCap - 1)] = (int32_t)i;
      qn = __builtin_amdgcn_readfirstlane(qn + np + __popcll(bs));
      while (qn >= 32) critic_queue(32);
      continue;
    }
    // ---- next_obs: base + critic only (get_values, ppo.py:84-89)
    x[0] = load_x0_obs(a.next_obs + ic * a.D, a.D, a.nq1, valid, h, a.q4);
    dense1_tanh(y, lds + L.W1, L.S1, lds + L.b1, x[0], a.nq1, l31, h);
    dense_tanh(x, lds + L.W2, lds + L.b2, y, l31, h);
    dense_tanh(y, lds + L.Wc, lds + L.bc, x, l31, h);
    const float nv = value_head(lds + L.Wv, bv, y, h);
    if (valid && h == 0) {
      a.logp[i] = logp;
      a.values[i] = v;
      a.next_values[i] = nv;
    }
  }
  if (a.row > 0) {
    // the waves' remainders (< 32 each) pooled across the workgroup and run as full tiles: one
    // partial critic tile per wave at the end was ~8 % more MFMA work than the queued samples need
    int* rem = (int*)lds_ + L.queue + kWaves * kQueueCap;  // [kWaves] counts, [kWaves] heads
    if (lane == 0) {
      rem[wave] = qn;
      rem[kWaves + wave] = qh;
    }
    __syncthreads();
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += rem[w];
    if (32 * wave < tot) {
      const int pos = 32 * wave + l31;
      bool qv = pos < tot;
      int64_t k = 0;
      if (qv) {
        int base = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
          const int c = rem[w];
          if (pos >= base && pos < base + c)
            k = ((const int32_t*)lds_)[L.queue + w * kQueueCap +
                                       ((rem[kWaves + w] + pos - base) & (kQueueCap - 1))];
          base += c;
        }
      }
      critic_tile(qv, k);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Action sampling for the rollout (get_actions, ppo.py:73-82 / continuous_ppo.py:83-93): base +
// actor forward, then Categorical(logits).sample() or Normal(mean, exp(log_std)).sample() on the
// lane that holds the sample.  Randomness: Philox4x32-10 keyed by `seed`, counter (sample index,
// call counter) -- a deterministic stream of its own (the reference draws from torch's generator:
// same distribution, not the same draws).
__device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * b) >> 32);
}

__device__ __forceinline__ void philox4x32(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = mulhi32(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    c[0] = hi1 ^ c[1] ^ k0;
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k1;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// u32 -> uniform in (0, 1): 24 random bits, centred in their interval (never 0 or 1)
__device__ __forceinline__ float u01(uint32_t x) {
  return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

struct ActArgs {
  LdsLayout L;
  ParamOffsets po;
  const float* params;
  const float* obs;
  void* actions;   // sampled actions, or null (heads only)
  float* heads;    // optional [n][A]: the logits / Gaussian means the samples are drawn from
  // optional [n][A] (continuous): the environment's action for each Gaussian sample u --
  // tanh(u) (squash 1) or low + (tanh(u) + 1) * (high - low) / 2 (squash 2)
  float* env_act;
  int squash;
  float sq_lo[16], sq_half[16];
  int64_t n;
  uint32_t seed_lo, seed_hi, ctr_lo, ctr_hi;
  int D, D8, nq1, A;
  int q4;
};

__device__ __forceinline__ void load_weights_actor(float* lds, const ActArgs& a, int tid) {
  const float* P = a.params;
  const LdsLayout& L = a.L;
  for (int k = tid; k < H * L.S1; k += kThreads) {
    const int o = k / L.S1, c = k % L.S1;
    lds[L.W1 + k] = c < a.D ? P[a.po.W1 + o * a.D + c] * kTS : 0.0f;
  }
  for (int k = tid; k < H * H; k += kThreads) {
    const int o = k >> 6, c = k & 63;
    lds[L.W2 + o * SW + c] = P[a.po.W2 + k] * kTS;
    lds[L.Wa + o * SW + c] = P[a.po.Wa + k] * kTS;
  }
  for (int k = tid; k < a.A * H; k += kThreads) lds[L.Wo + k] = P[a.po.Wo + k];
  for (int k = tid; k < H; k += kThreads) {
    lds[L.b1 + k] = P[a.po.b1 + k] * kTS;
    lds[L.b2 + k] = P[a.po.b2 + k] * kTS;
    lds[L.ba + k] = P[a.po.ba + k] * kTS;
  }
  for (int k = tid; k < 32; k += kThreads) {
    lds[L.bo + k] = k < a.A ? P[a.po.bo + k] : 0.0f;
    lds[L.ls + k] = (a.po.ls >= 0 && k < a.A) ? P[a.po.ls + k] : 0.0f;
  }
}

template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 4) void act_kernel(ActArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  load_weights_actor(lds_, a, tid);
  __syncthreads();
  const LdsLayout& L = a.L;
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles;
       tile += (int64_t)gridDim.x * kWaves) {
    float* lds = opaque_base(lds_);
    const int64_t i = tile * 32 + l31;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : 0;
    f32x16 x[2], y[2];
    x[0] = load_x0_obs(a.obs + ic * a.D, a.D, a.nq1, valid, h, a.q4);
    dense1_tanh(y, lds + L.W1, L.S1, lds + L.b1, x[0], a.nq1, l31, h);       // y = h1
    dense_tanh(x, lds + L.W2, lds + L.b2, y, l31, h);                         // x = h2
    dense_tanh(y, lds + L.Wa, lds + L.ba, x, l31, h);                         // y = actor hidden
    float out[AMAX];
    heads<AMAX>(out, lds + L.Wo, lds + L.bo, a.A, y, h);
    if (!valid || h != 0) continue;
    if (a.heads) {
#pragma unroll
      for (int k = 0; k < AMAX; ++k)
        if (k < a.A) a.heads[i * a.A + k] = out[k];
    }
    if (!a.actions) continue;
    if (CONT) {
      // Normal(mean, exp(log_std)).sample(): Box-Muller pairs from Philox (4 uniforms per call)
      float* act = (float*)a.actions + i * a.A;
#pragma unroll
      for (int k0 = 0; k0 < AMAX; k0 += 4) {
        if (k0 < a.A) {
          uint32_t c[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32) ^ (uint32_t)(k0 << 24),
                           a.ctr_lo, a.ctr_hi};
          philox4x32(c, a.seed_lo, a.seed_hi);
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const float r = sqrtf(-2.0f * __logf(u01(c[2 * p])));
            float sn, cs;
            __sincosf(6.28318530717958647692f * u01(c[2 * p + 1]), &sn, &cs);
            const int k = k0 + 2 * p;
            const float u0 = k < AMAX ? out[k] + __expf(lds[L.ls + k]) * (r * cs) : 0.f;
            const float u1 = k + 1 < AMAX ? out[k + 1] + __expf(lds[L.ls + k + 1]) * (r * sn) : 0.f;
            if (k < a.A) act[k] = u0;
            if (k + 1 < a.A) act[k + 1] = u1;
            if (a.env_act) {
              // the squashed env action (SURVEY 8 f2 extension; the reference samples the raw
              // Gaussian, continuous_ppo.py:83-93): accurate tanhf, not the MLP's fast form
              float* env = a.env_act + i * a.A;
              if (k < a.A) {
                const float t0 = tanhf(u0);
                env[k] = a.squash == 2 ? a.sq_lo[k] + (t0 + 1.0f) * a.sq_half[k] : t0;
              }
              if (k + 1 < a.A) {
                const float t1 = tanhf(u1);
                env[k + 1] = a.squash == 2 ? a.sq_lo[k + 1] + (t1 + 1.0f) * a.sq_half[k + 1] : t1;
              }
            }
          }
        }
      }
    } else {
      // Categorical(logits).sample() by inverse CDF on one uniform
      uint32_t c[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), a.ctr_lo, a.ctr_hi};
      philox4x32(c, a.seed_lo, a.seed_hi);
      float mx = out[0];
#pragma unroll
      for (int k = 1; k < AMAX; ++k)
        if (k < a.A) mx = fmaxf(mx, out[k]);
      float e[AMAX], se = 0.0f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        e[k] = k < a.A ? __expf(out[k] - mx) : 0.0f;
        se += e[k];
      }
      // the first k whose cumulative mass exceeds u * sum (the last action takes the remainder)
      const float target = u01(c[0]) * se;
      int pick = a.A - 1;
      float cum = 0.0f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        if (k < a.A - 1) {
          cum += e[k];
          if (pick == a.A - 1 && target < cum) pick = k;
        }
      }
      ((int32_t*)a.actions)[i] = pick;
    }
  }
}

KArgs base_args(const MlpShape& sh, const ParamOffsets& po, const float* params) {
  KArgs k{};
  k.L = make_layout(sh);
  k.po = po;
  k.params = params;
  k.D = sh.D;
  k.D8 = sh.D8;
  k.nq1 = sh.D8 / 8;
  k.A = sh.A;
  k.R = sh.R;
  return k;
}

#define DPPO_DISPATCH(KERNEL, SH, GRID, LDSB, STREAM, ARGS)                                    \
  do {                                                                                       \
    const int A_ = (SH).A;                                                                   \
    const bool C_ = (SH).continuous != 0;                                                    \
    if (A_ <= 2) {                                                                           \
      if (C_) DPPO_LAUNCH((KERNEL<2, true>), GRID, dim3(kThreads), LDSB, STREAM, ARGS); \
      else DPPO_LAUNCH((KERNEL<2, false>), GRID, dim3(kThreads), LDSB, STREAM, ARGS);   \
    } else if (A_ <= 4) {                                                                    \
      if (C_) DPPO_LAUNCH((KERNEL<4, true>), GRID, dim3(kThreads), LDSB, STREAM, ARGS); \
      else DPPO_LAUNCH((KERNEL<4, false>), GRID, dim3(kThreads), LDSB, STREAM, ARGS);   \
    } else if (A_ <= 8) {                                                                    \
      if (C_) DPPO_LAUNCH((KERNEL<8, true>), GRID, dim3(kThreads), LDSB, STREAM, ARGS); \
      else DPPO_LAUNCH((KERNEL<8, false>), GRID, dim3(kThreads), LDSB, STREAM, ARGS);   \
    } else {                                                                                 \
      if (C_) DPPO_LAUNCH((KERNEL<16, true>), GRID, dim3(kThreads), LDSB, STREAM, ARGS); \
      else DPPO_LAUNCH((KERNEL<16, false>), GRID, dim3(kThreads), LDSB, STREAM, ARGS);  \
    }                                                                                        \
  } while (0)

void raise_lds_limits() {
  static const bool done = [] {
#define DPPO_SET(A, C) raise_dyn_lds((const void*)eval_kernel<A, C>);
    DPPO_SET(2, false) DPPO_SET(2, true) DPPO_SET(4, false) DPPO_SET(4, true)
    DPPO_SET(8, false) DPPO_SET(8, true) DPPO_SET(16, false) DPPO_SET(16, true)
#undef DPPO_SET
#define DPPO_SET(A, C) raise_dyn_lds((const void*)act_kernel<A, C>);
    DPPO_SET(2, false) DPPO_SET(2, true) DPPO_SET(4, false) DPPO_SET(4, true)
    DPPO_SET(8, false) DPPO_SET(8, true) DPPO_SET(16, false) DPPO_SET(16, true)
#undef DPPO_SET
    return true;
  }();
  (void)done;
}

int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  return cus;
}

}  // namespace

size_t mlp_lds_bytes_eval(const MlpShape& sh) {
  const LdsLayout L = make_layout(sh);
  return (size_t)L.total * sizeof(float);
}

int launch_eval(const MlpShape& sh, const ParamOffsets& po, const float* params, const float* obs,
                const void* actions, const float* next_obs, float* logp, float* values,
                float* next_values, int64_t n, hipStream_t s, EvalReuse* reuse) {
  if (n <= 0) return DPPO_OK;
  KArgs k = base_args(sh, po, params);
  if (reuse && reuse->row > 0 && reuse->row < n) k.row = reuse->row;
  k.obs = obs;
  k.actions = actions;
  k.next_obs = next_obs;
  k.q4 = (sh.D % 4 == 0) && ((uintptr_t)obs % 16 == 0) && (!next_obs || (uintptr_t)next_obs % 16 == 0);
  k.logp = logp;
  k.values = values;
  k.next_values = next_values;
  k.n = n;
  const size_t lds = (size_t)k.L.total * sizeof(float);
  raise_lds_limits();
  // persistent: two workgroups per CU (their LDS weight images fill it), grid-stride over tiles
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  const int64_t ntiles = (n + 31) / 32;
  int64_t g = (ntiles + kWaves - 1) / kWaves;
  if (g > 2 * cus) g = 2 * cus;
  DPPO_DISPATCH(eval_kernel, sh, dim3((unsigned)g), lds, s, k);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_act(const MlpShape& sh, const ParamOffsets& po, const float* params, const float* obs,
               void* actions, int64_t n, uint64_t seed, uint64_t counter, hipStream_t s,
               float* heads, const ActSquash* squash) {
  if (n <= 0) return DPPO_OK;
  ActArgs k{};
  if (squash && squash->env_actions) {
    if (!sh.continuous || sh.A > 16) {
      set_error("tanh squash needs a continuous action space of at most 16 dims");
      return DPPO_EINVAL;
    }
    k.env_act = squash->env_actions;
    k.squash = squash->low && squash->high ? 2 : 1;
    for (int j = 0; j < sh.A && k.squash == 2; ++j) {
      k.sq_lo[j] = squash->low[j];
      k.sq_half[j] = 0.5f * (squash->high[j] - squash->low[j]);
    }
  }
  k.L = make_layout(sh);
  k.po = po;
  k.params = params;
  k.obs = obs;
  k.actions = actions;
  k.heads = heads;
  k.n = n;
  k.seed_lo = (uint32_t)seed;
  k.seed_hi = (uint32_t)(seed >> 32);
  k.ctr_lo = (uint32_t)counter;
  k.ctr_hi = (uint32_t)(counter >> 32);
  k.D = sh.D;
  k.D8 = sh.D8;
  k.nq1 = sh.D8 / 8;
  k.A = sh.A;
  k.q4 = (sh.D % 4 == 0) && ((uintptr_t)obs % 16 == 0);
  const size_t lds = (size_t)k.L.total * sizeof(float);
  raise_lds_limits();
  const int64_t ntiles = (n + 31) / 32;
  int64_t g = (ntiles + kWaves - 1) / kWaves;
  if (g > 2 * cu_count()) g = 2 * cu_count();
  DPPO_DISPATCH(act_kernel, sh, dim3((unsigned)g), lds, s, k);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
