// Default actor-critic MLP (hidden 64) on gfx950 fp32 MFMA: old-policy evaluation and the fused
// minibatch {gather, forward, loss, analytic backward, weight-gradient} kernel.
//
// Reference: ActorCriticNetwork (diamond/ppo.py:40-96), ContinuousActorCriticNetwork
// (diamond/continuous_ppo.py:50-111), old-policy eval (ppo.py:235-238), minibatch loss
// (ppo.py:261-280, continuous_ppo.py:273-292) and loss.backward() (ppo.py:283).
//
// ---- Tiling -----------------------------------------------------------------------------------
// Activations are FEATURE-major: a [64 features x 32 samples] activation is two 32x32 MFMA
// accumulator tiles (f32x16 per lane) of v_mfma_f32_32x32x2_f32, sample on the lane
// (col = lane & 31), features in the 16 registers (row = (r&3) + 8(r>>2) + 4(lane>>5)).
// A layer Y = W X + b then sums over X's ROW index, so X's accumulator registers ARE the next
// MFMA's B operand with no data movement (k-step r uses rows krow(r,0) and krow(r,1) = +4);
// the A operand is the matching W element, read from an LDS image of W (row stride 68 floats:
// conflict-free for both the forward ds_read_b128 of W[o][k..k+3] and the backward ds_read_b32
// of W[k][i..i+31]).  The input gradient dX = W^T dZ chains the same way.  Only the weight
// gradients dW = dZ X^T sum over the lane (sample) index; for those dZ and X are staged through a
// per-wave LDS image [sample][feature] and read back as MFMA operands with the sample in the k
// slot.  All math is exact fp32 (f32-input MFMA = an ordered fmaf chain, no xf32 on gfx950).
//
// ---- Work decomposition -----------------------------------------------------------------------
// One 256-thread workgroup per CU (LDS: the weights once per workgroup + two 8.5 KiB staging
// images per wave).  Each wave walks a fixed, static list of 32-sample tiles and keeps its
// weight-gradient accumulators (224 fp32 registers per lane: dW1, dW2, dWa, dWc) live across
// tiles; heads, biases and log-std gradients are per-lane scalars.  At the end the four waves'
// partial gradients are summed through LDS in a fixed order and written as ONE slab per
// workgroup; optim.hip sums the slabs in a fixed order (bit-reproducible, no float atomics).
#include "common.h"

namespace dppo {
namespace {

constexpr int H = 64;
constexpr int SW = H + 4;  // LDS row stride (floats) of H-wide weight images and staging images
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
constexpr float kHalfLog2PiPlusHalf = 1.41893853320467274178f;  // 0.5 + 0.5 log(2 pi)

struct LdsLayout {
  int W1, S1;          // W1 image [H][S1], S1 = D8 + 4 (zero-padded columns D..S1)
  int W2, Wa, Wc;      // [H][SW]
  int Wo;              // [A][H]  (logits or mean head)
  int Wv;              // [H]
  int b1, b2, ba, bc;  // [H]
  int bo, ls;          // [32]
  int bv;              // [4]
  int stage;           // per-wave staging: 2 x [32][SW]
  int weights_end;
  int total;           // floats
};

struct KArgs {
  LdsLayout L;
  ParamOffsets po;
  const float* params;
  // grad kernel
  const float* rec;
  const int32_t* idx;
  int m;
  float inv_m, clip_eps, vf, ent;
  float* slabs;
  int64_t slab_stride, p_total;
  // eval kernel
  const float* obs;
  const void* actions;
  const float* next_obs;
  float *logp, *values, *next_values;
  int64_t n;
  // shapes
  int D, D8, nq1, A, R;
};

__host__ __device__ inline int align4(int x) { return (x + 3) & ~3; }

LdsLayout make_layout(const MlpShape& sh, bool staging) {
  LdsLayout L{};
  int o = 0;
  L.S1 = sh.D8 + 4;
  L.W1 = o; o += align4(H * L.S1);
  L.W2 = o; o += H * SW;
  L.Wa = o; o += H * SW;
  L.Wc = o; o += H * SW;
  L.Wo = o; o += align4(sh.A * H);
  L.Wv = o; o += H;
  L.b1 = o; o += H;
  L.b2 = o; o += H;
  L.ba = o; o += H;
  L.bc = o; o += H;
  L.bo = o; o += 32;
  L.ls = o; o += 32;
  L.bv = o; o += 4;
  L.weights_end = o;
  L.stage = o;
  if (staging) o += kWaves * 2 * 32 * SW;
  L.total = o;
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
    lds[L.W1 + k] = c < a.D ? P[a.po.W1 + o * a.D + c] : 0.0f;
  }
  for (int k = tid; k < H * H; k += kThreads) {
    const int o = k >> 6, c = k & 63;
    lds[L.W2 + o * SW + c] = P[a.po.W2 + k];
    lds[L.Wa + o * SW + c] = P[a.po.Wa + k];
    lds[L.Wc + o * SW + c] = P[a.po.Wc + k];
  }
  for (int k = tid; k < a.A * H; k += kThreads) lds[L.Wo + k] = P[a.po.Wo + k];
  for (int k = tid; k < H; k += kThreads) {
    lds[L.Wv + k] = P[a.po.Wv + k];
    lds[L.b1 + k] = P[a.po.b1 + k];
    lds[L.b2 + k] = P[a.po.b2 + k];
    lds[L.ba + k] = P[a.po.ba + k];
    lds[L.bc + k] = P[a.po.bc + k];
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

__device__ __forceinline__ void tanh_inplace(f32x16& x) {
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 1.0f - 2.0f / (1.0f + __expf(2.0f * x[r]));
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

// dx[ib] (+)= sum_ob W[ob-rows][ib-cols]^T dz[ob]   (W: [64 out][64 in] image, stride SW)
__device__ __forceinline__ void dense_T(f32x16 (&dx)[2], const float* W, const f32x16 (&dz)[2],
                                        int l31, int h, bool accumulate) {
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
    f32x16 acc;
    if (accumulate) {
      acc = dx[ib];
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    }
    const float* wp = W + 4 * h * SW + ib * 32 + l31;
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = ob * 32 + (r & 3) + 8 * (r >> 2);
        acc = mfma(wp[k * SW], dz[ob][r], acc);
      }
    }
    dx[ib] = acc;
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Stage a feature-major block into a [sample][feature] LDS image (stride SW).
__device__ __forceinline__ void stage(float* S, const f32x16& v, int fb, int l31, int h) {
  float* p = S + l31 * SW + fb * 32 + 4 * h;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 w;
    w[0] = v[4 * q + 0];
    w[1] = v[4 * q + 1];
    w[2] = v[4 * q + 2];
    w[3] = v[4 * q + 3];
    *(f32x4*)(p + 8 * q) = w;
  }
}

__device__ __forceinline__ f32x16 unstage(const float* S, int fb, int l31, int h) {
  f32x16 v;
  const float* p = S + l31 * SW + fb * 32 + 4 * h;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 w = *(const f32x4*)(p + 8 * q);
    v[4 * q + 0] = w[0];
    v[4 * q + 1] = w[1];
    v[4 * q + 2] = w[2];
    v[4 * q + 3] = w[3];
  }
  return v;
}

// dW[ob][ib] += sum over the 32 staged samples of SZ[s][ob*32+.] (x) SX[s][ib*32+.]
template <int NIB>
__device__ __forceinline__ void wgrad(f32x16 (&acc)[2][2], const float* SZ, const float* SX,
                                      int l31, int h) {
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int row = (2 * t + h) * SW;
    const float a0 = SZ[row + l31];
    const float a1 = SZ[row + 32 + l31];
    const float b0 = SX[row + l31];
    acc[0][0] = mfma(a0, b0, acc[0][0]);
    acc[1][0] = mfma(a1, b0, acc[1][0]);
    if (NIB == 2) {
      const float b1 = SX[row + 32 + l31];
      acc[0][1] = mfma(a0, b1, acc[0][1]);
      acc[1][1] = mfma(a1, b1, acc[1][1]);
    }
    if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
}

// Column sum of a staged [32][SW] image for this lane's feature (lane = feature 0..63).
__device__ __forceinline__ float colsum(const float* S, int lane) {
  float s = 0.0f;
#pragma unroll 8
  for (int r = 0; r < 32; ++r) s += S[r * SW + lane];
  return s;
}

__device__ __forceinline__ void one_minus_sq_mul(f32x16& d, const f32x16& y) {
#pragma unroll
  for (int r = 0; r < 16; ++r) d[r] = d[r] * (1.0f - y[r] * y[r]);
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
      const float* wp = Wo + a * H + 4 * h;
#pragma unroll
      for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 w = *(const f32x4*)(wp + fb * 32 + 8 * q);
          part += w[0] * x[fb][4 * q + 0] + w[1] * x[fb][4 * q + 1] + w[2] * x[fb][4 * q + 2] +
                  w[3] * x[fb][4 * q + 3];
        }
    }
    out[a] = part + __shfl_xor(part, 32) + bo[a];
  }
}

__device__ __forceinline__ float value_head(const float* Wv, float bv, const f32x16 (&x)[2],
                                            int h) {
  float part = 0.0f;
  const float* wp = Wv + 4 * h;
#pragma unroll
  for (int fb = 0; fb < 2; ++fb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 w = *(const f32x4*)(wp + fb * 32 + 8 * q);
      part += w[0] * x[fb][4 * q + 0] + w[1] * x[fb][4 * q + 1] + w[2] * x[fb][4 * q + 2] +
              w[3] * x[fb][4 * q + 3];
    }
  return part + __shfl_xor(part, 32) + bv;
}

// dx[fb][r] = sum_a Wo[a][f(fb, r)] * g[a]   (head input gradient, VALU)
template <int AMAX>
__device__ __forceinline__ void heads_T(f32x16 (&dx)[2], const float* Wo, int A,
                                        const float (&g)[AMAX], int h) {
#pragma unroll
  for (int fb = 0; fb < 2; ++fb)
#pragma unroll
    for (int r = 0; r < 16; ++r) dx[fb][r] = 0.0f;
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    if (a < A) {
      const float* wp = Wo + a * H + 4 * h;
#pragma unroll
      for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 w = *(const f32x4*)(wp + fb * 32 + 8 * q);
          dx[fb][4 * q + 0] += w[0] * g[a];
          dx[fb][4 * q + 1] += w[1] * g[a];
          dx[fb][4 * q + 2] += w[2] * g[a];
          dx[fb][4 * q + 3] += w[3] * g[a];
        }
    }
  }
}

// Load the layer-1 input block (zero-padded to 32 features) for one sample row.
__device__ __forceinline__ f32x16 load_x0_rec(const float* rec, int nq1, int h) {
  f32x16 x;
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < nq1) {
      const f32x4 w = *(const f32x4*)(rec + 8 * q + 4 * h);
      x[4 * q + 0] = w[0];
      x[4 * q + 1] = w[1];
      x[4 * q + 2] = w[2];
      x[4 * q + 3] = w[3];
    }
  }
  return x;
}

__device__ __forceinline__ f32x16 load_x0_obs(const float* o, int D, int nq1, bool valid, int h) {
  f32x16 x;
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = 0.0f;
  if (valid) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < nq1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f = 8 * q + 4 * h + j;
          x[4 * q + j] = f < D ? o[f] : 0.0f;
        }
      }
    }
  }
  return x;
}

// ------------------------------------------------------------------------------------------------
// Old-policy evaluation (ppo.py:235-238): one wave per 32-sample tile, grid-stride over tiles.
template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 2) void eval_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  load_weights(lds_, a, tid);
  __syncthreads();
  const LdsLayout& L = a.L;
  const float bv = lds_[L.bv];
  const int64_t ntiles = (a.n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + wave; tile < ntiles;
       tile += (int64_t)gridDim.x * kWaves) {
    float* lds = opaque_base(lds_);
    const int64_t i = tile * 32 + l31;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : 0;
    // ---- obs: full actor-critic forward
    f32x16 x0 = load_x0_obs(a.obs + ic * a.D, a.D, a.nq1, valid, h);
    f32x16 h1[2], h2[2], ha[2], hc[2];
    dense1_tanh(h1, lds + L.W1, L.S1, lds + L.b1, x0, a.nq1, l31, h);
    dense_tanh(h2, lds + L.W2, lds + L.b2, h1, l31, h);
    dense_tanh(ha, lds + L.Wa, lds + L.ba, h2, l31, h);
    dense_tanh(hc, lds + L.Wc, lds + L.bc, h2, l31, h);
    float out[AMAX];
    heads<AMAX>(out, lds + L.Wo, lds + L.bo, a.A, ha, h);
    const float v = value_head(lds + L.Wv, bv, hc, h);
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
      const int act = ((const int32_t*)a.actions)[ic];
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
    // ---- next_obs: base + critic only (get_values, ppo.py:84-89)
    x0 = load_x0_obs(a.next_obs + ic * a.D, a.D, a.nq1, valid, h);
    dense1_tanh(h1, lds + L.W1, L.S1, lds + L.b1, x0, a.nq1, l31, h);
    dense_tanh(h2, lds + L.W2, lds + L.b2, h1, l31, h);
    dense_tanh(hc, lds + L.Wc, lds + L.bc, h2, l31, h);
    const float nv = value_head(lds + L.Wv, bv, hc, h);
    if (valid && h == 0) {
      a.logp[i] = logp;
      a.values[i] = v;
      a.next_values[i] = nv;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Fused minibatch step (ppo.py:261-283): gather -> forward -> loss -> backward -> dW partials.
template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 1) void grad_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const LdsLayout& L = a.L;
  load_weights(lds_, a, tid);
  __syncthreads();
  const float bv = lds_[L.bv];

  f32x16 gW1[2], gW2[2][2], gWa[2][2], gWc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) gW1[i][r] = 0.0f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) gW2[i][j][r] = gWa[i][j][r] = gWc[i][j][r] = 0.0f;
  }
  float gWo[AMAX];
#pragma unroll
  for (int k = 0; k < AMAX; ++k) gWo[k] = 0.0f;
  float gWv = 0.f, gb1 = 0.f, gb2 = 0.f, gba = 0.f, gbc = 0.f, gbh = 0.f;
  float s_pi = 0.f, s_v = 0.f, s_ent = 0.f;

  const int ntiles = (a.m + 31) / 32;
  for (int tile = blockIdx.x * kWaves + wave; tile < ntiles; tile += gridDim.x * kWaves) {
    float* lds = opaque_base(lds_);
    float* SX = lds + L.stage + wave * (2 * 32 * SW);
    float* SZ = SX + 32 * SW;
    const float* Wo = lds + L.Wo;
    const int si = tile * 32 + l31;
    const bool valid = si < a.m;
    const int64_t gi = a.idx[valid ? si : 0];
    const float* rec = a.rec + gi * a.R;

    // ---------------- forward
    f32x16 h1[2], h2[2], ha[2], hc[2];
    {
      const f32x16 x0 = load_x0_rec(rec, a.nq1, h);
      dense1_tanh(h1, lds + L.W1, L.S1, lds + L.b1, x0, a.nq1, l31, h);
    }
    dense_tanh(h2, lds + L.W2, lds + L.b2, h1, l31, h);
    dense_tanh(ha, lds + L.Wa, lds + L.ba, h2, l31, h);
    dense_tanh(hc, lds + L.Wc, lds + L.bc, h2, l31, h);
    float out[AMAX];
    heads<AMAX>(out, Wo, lds + L.bo, a.A, ha, h);
    const float v = value_head(lds + L.Wv, bv, hc, h);

    // ---------------- loss + d loss / d outputs (Appendix A.3-A.4 of SURVEY.md)
    const f32x4 sc = *(const f32x4*)(rec + a.D8);  // {action bits, old logp, adv, return}
    const float adv = sc[2], ret = sc[3];
    float logp, ent;
    float p[AMAX], lp[AMAX];
    float xa[AMAX], sig[AMAX];
    if (CONT) {
      logp = 0.f;
      ent = 0.f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        xa[k] = 0.f;
        sig[k] = 1.f;
        if (k < a.A) {
          xa[k] = rec[a.D8 + 4 + k];
          const float ls = lds[L.ls + k];
          sig[k] = expf(ls);
          const float lsc = logf(sig[k]);
          const float d = xa[k] - out[k];
          logp += -(d * d) / (2.0f * (sig[k] * sig[k])) - lsc - kLogSqrt2Pi;
          ent += kHalfLog2PiPlusHalf + lsc;
        }
      }
    } else {
      const int act = __float_as_int(sc[0]);
      float mx = out[0];
#pragma unroll
      for (int k = 1; k < AMAX; ++k)
        if (k < a.A) mx = fmaxf(mx, out[k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k)
        if (k < a.A) se += expf(out[k] - mx);
      const float lse = mx + logf(se);
      logp = 0.f;
      ent = 0.f;
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        lp[k] = 0.f;
        p[k] = 0.f;
        if (k < a.A) {
          lp[k] = out[k] - lse;
          p[k] = expf(lp[k]);
          ent -= p[k] * lp[k];
          if (k == act) logp = lp[k];
        }
      }
    }
    const float ratio = expf(logp - sc[1]);                         // ppo.py:266
    const float rcl = fminf(fmaxf(ratio, 1.0f - a.clip_eps), 1.0f + a.clip_eps);
    const float u = -adv * ratio, w = -adv * rcl;                   // ppo.py:267-269
    const float inr = (ratio >= 1.0f - a.clip_eps && ratio <= 1.0f + a.clip_eps) ? 1.f : 0.f;
    const float gu = u > w ? 1.f : (u == w ? 0.5f : 0.f);           // torch maximum ties split
    const float gw = w > u ? 1.f : (u == w ? 0.5f : 0.f);
    const float vm = valid ? a.inv_m : 0.f;
    const float dlogp = (gu * -adv + gw * -adv * inr) * vm * ratio;
    const float dv = a.vf * (v - ret) * vm;                          // ppo.py:272
    if (valid && h == 0) {
      s_pi += fmaxf(u, w);
      s_v += 0.5f * (v - ret) * (v - ret);
      s_ent += ent;
    }
    float dout[AMAX], dls[AMAX];
#pragma unroll
    for (int k = 0; k < AMAX; ++k) {
      dout[k] = 0.f;
      dls[k] = 0.f;
      if (k < a.A) {
        if (CONT) {
          const float dd = xa[k] - out[k];
          const float z = dd / sig[k];
          dout[k] = dlogp * dd / (sig[k] * sig[k]);
          dls[k] = dlogp * (z * z - 1.0f);
        } else {
          const int act = __float_as_int(sc[0]);
          dout[k] = dlogp * ((k == act ? 1.f : 0.f) - p[k]) +
                    a.ent * vm * p[k] * (lp[k] + ent);
        }
      }
    }

    // ---------------- head gradients (VALU over staged samples)
    // SX <- {dout[0..A), dv at col 32, dls at cols 33..}, SZ <- ha
    if (h == 0) {
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        SX[l31 * SW + k] = dout[k];
        if (CONT) SX[l31 * SW + 33 + k] = dls[k];
      }
      SX[l31 * SW + 32] = dv;
    }
    stage(SZ, ha[0], 0, l31, h);
    stage(SZ, ha[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
#pragma unroll 4
    for (int s = 0; s < 32; ++s) {
      const float x = SZ[s * SW + lane];
#pragma unroll
      for (int k = 0; k < AMAX; ++k)
        if (k < a.A) gWo[k] += SX[s * SW + k] * x;
    }
    gbh += colsum(SX, lane);  // lanes < A: bo, lane 32: bv, lanes 33..: log_std terms
    __builtin_amdgcn_wave_barrier();
    stage(SZ, hc[0], 0, l31, h);
    stage(SZ, hc[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
#pragma unroll 8
    for (int s = 0; s < 32; ++s) gWv += SX[s * SW + 32] * SZ[s * SW + lane];
    __builtin_amdgcn_wave_barrier();

    // dZa = (Wo^T dout) (1 - ha^2) ; dZc = (Wv dv) (1 - hc^2)
    f32x16 dza[2], dzc[2];
    heads_T<AMAX>(dza, Wo, a.A, dout, h);
    one_minus_sq_mul(dza[0], ha[0]);
    one_minus_sq_mul(dza[1], ha[1]);
    {
      const float* wp = lds + L.Wv + 4 * h;
#pragma unroll
      for (int fb = 0; fb < 2; ++fb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 wv = *(const f32x4*)(wp + fb * 32 + 8 * q);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float y = hc[fb][4 * q + j];
            dzc[fb][4 * q + j] = wv[j] * dv * (1.0f - y * y);
          }
        }
    }

    // ---------------- dWa, dWc  (input h2)
    stage(SX, h2[0], 0, l31, h);
    stage(SX, h2[1], 1, l31, h);
    stage(SZ, dza[0], 0, l31, h);
    stage(SZ, dza[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
    wgrad<2>(gWa, SZ, SX, l31, h);
    gba += colsum(SZ, lane);
    __builtin_amdgcn_wave_barrier();
    stage(SZ, dzc[0], 0, l31, h);
    stage(SZ, dzc[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
    wgrad<2>(gWc, SZ, SX, l31, h);
    gbc += colsum(SZ, lane);

    // ---------------- dh2 = Wa^T dZa + Wc^T dZc ; dZ2 = dh2 (1 - h2^2)
    f32x16 dz2[2];
    dense_T(dz2, lds + L.Wa, dza, l31, h, false);
    dense_T(dz2, lds + L.Wc, dzc, l31, h, true);
    one_minus_sq_mul(dz2[0], unstage(SX, 0, l31, h));  // h2, still staged in SX
    one_minus_sq_mul(dz2[1], unstage(SX, 1, l31, h));
    __builtin_amdgcn_wave_barrier();

    // ---------------- dW2 (input h1)
    stage(SX, h1[0], 0, l31, h);
    stage(SX, h1[1], 1, l31, h);
    stage(SZ, dz2[0], 0, l31, h);
    stage(SZ, dz2[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
    wgrad<2>(gW2, SZ, SX, l31, h);
    gb2 += colsum(SZ, lane);

    // ---------------- dZ1 = (W2^T dZ2) (1 - h1^2) ; dW1 (input x0)
    f32x16 dz1[2];
    dense_T(dz1, lds + L.W2, dz2, l31, h, false);
    one_minus_sq_mul(dz1[0], unstage(SX, 0, l31, h));  // h1, staged in SX for dW2
    one_minus_sq_mul(dz1[1], unstage(SX, 1, l31, h));
    __builtin_amdgcn_wave_barrier();
    {
      const f32x16 x0 = load_x0_rec(rec, a.nq1, h);
      stage(SX, x0, 0, l31, h);
    }
    stage(SZ, dz1[0], 0, l31, h);
    stage(SZ, dz1[1], 1, l31, h);
    __builtin_amdgcn_wave_barrier();
    {
      f32x16 g1[2][2];
      g1[0][0] = gW1[0];
      g1[1][0] = gW1[1];
      wgrad<1>(g1, SZ, SX, l31, h);
      gW1[0] = g1[0][0];
      gW1[1] = g1[1][0];
    }
    gb1 += colsum(SZ, lane);
    __builtin_amdgcn_wave_barrier();
  }

  // ---------------- epilogue: sum the four waves' partials through LDS, write one slab
  __syncthreads();
  float* acc = lds_;  // reuse: [p_total + 8]
  const int np = (int)a.p_total + 8;
  for (int k = tid; k < np; k += kThreads) acc[k] = 0.0f;
  __syncthreads();
  const ParamOffsets& po = a.po;
  // loss sums over the wave
  for (int off = 32; off >= 1; off >>= 1) {
    s_pi += __shfl_xor(s_pi, off);
    s_v += __shfl_xor(s_v, off);
    s_ent += __shfl_xor(s_ent, off);
  }
  for (int w = 0; w < kWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ob = 0; ob < 2; ++ob) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int o = ob * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
          for (int ib = 0; ib < 2; ++ib) {
            const int i = ib * 32 + l31;
            acc[po.W2 + o * H + i] += gW2[ob][ib][r];
            acc[po.Wa + o * H + i] += gWa[ob][ib][r];
            acc[po.Wc + o * H + i] += gWc[ob][ib][r];
          }
          if (l31 < a.D) acc[po.W1 + o * a.D + l31] += gW1[ob][r];
        }
      }
#pragma unroll
      for (int k = 0; k < AMAX; ++k)
        if (k < a.A) acc[po.Wo + k * H + lane] += gWo[k];
      acc[po.Wv + lane] += gWv;
      acc[po.b1 + lane] += gb1;
      acc[po.b2 + lane] += gb2;
      acc[po.ba + lane] += gba;
      acc[po.bc + lane] += gbc;
      if (lane < a.A) acc[po.bo + lane] += gbh;
      if (lane == 32) acc[po.bv] += gbh;
      if (CONT && lane >= 33 && lane < 33 + a.A) acc[po.ls + (lane - 33)] += gbh;
      if (lane == 0) {
        acc[a.p_total + 0] += s_pi;
        acc[a.p_total + 1] += s_v;
        acc[a.p_total + 2] += s_ent;
      }
    }
    __syncthreads();
  }
  float* slab = a.slabs + (int64_t)blockIdx.x * a.slab_stride;
  for (int k = tid; k < np; k += kThreads) slab[k] = acc[k];
}

KArgs base_args(const MlpShape& sh, const ParamOffsets& po, const float* params, bool staging) {
  KArgs k{};
  k.L = make_layout(sh, staging);
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

void raise_lds_limits(const MlpShape& sh, size_t eval_b, size_t grad_b) {
  static bool done = false;
  if (done) return;
  done = true;
  const size_t mx = 160 * 1024;
  (void)eval_b;
  (void)grad_b;
#define DPPO_SET(A, C)                                                                  \
  (void)hipFuncSetAttribute((const void*)eval_kernel<A, C>,                             \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)mx);       \
  (void)hipFuncSetAttribute((const void*)grad_kernel<A, C>,                             \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)mx);
  DPPO_SET(2, false) DPPO_SET(2, true) DPPO_SET(4, false) DPPO_SET(4, true)
  DPPO_SET(8, false) DPPO_SET(8, true) DPPO_SET(16, false) DPPO_SET(16, true)
#undef DPPO_SET
  (void)sh;
}

}  // namespace

size_t mlp_lds_bytes_grad(const MlpShape& sh) {
  const LdsLayout L = make_layout(sh, true);
  return (size_t)L.total * sizeof(float);
}

size_t mlp_lds_bytes_eval(const MlpShape& sh) {
  const LdsLayout L = make_layout(sh, false);
  return (size_t)L.total * sizeof(float);
}

int launch_eval(const MlpShape& sh, const ParamOffsets& po, const float* params, const float* obs,
                const void* actions, const float* next_obs, float* logp, float* values,
                float* next_values, int64_t n, hipStream_t s) {
  if (n <= 0) return DPPO_OK;
  KArgs k = base_args(sh, po, params, false);
  k.obs = obs;
  k.actions = actions;
  k.next_obs = next_obs;
  k.logp = logp;
  k.values = values;
  k.next_values = next_values;
  k.n = n;
  const size_t lds = (size_t)k.L.total * sizeof(float);
  raise_lds_limits(sh, lds, mlp_lds_bytes_grad(sh));
  const int64_t ntiles = (n + 31) / 32;
  int64_t g = (ntiles + kWaves - 1) / kWaves;
  if (g > 1024) g = 1024;
  DPPO_DISPATCH(eval_kernel, sh, dim3((unsigned)g), lds, s, k);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int grad_grid(int32_t m) {
  const int ntiles = (m + 31) / 32;
  int g = (ntiles + kWaves - 1) / kWaves;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  return g;
}

int launch_grad(const MlpShape& sh, const ParamOffsets& po, const GradArgs& ga, int G,
                hipStream_t s) {
  KArgs k = base_args(sh, po, ga.params, true);
  k.rec = ga.rec;
  k.idx = ga.idx;
  k.m = ga.m;
  k.inv_m = ga.inv_m;
  k.clip_eps = ga.clip_eps;
  k.vf = ga.vf_coef;
  k.ent = ga.ent_coef;
  k.slabs = ga.slabs;
  k.slab_stride = ga.slab_stride;
  k.p_total = ga.p_total;
  const size_t lds_k = (size_t)k.L.total * sizeof(float);
  const size_t lds_acc = (size_t)(ga.p_total + 8) * sizeof(float);
  const size_t lds = lds_k > lds_acc ? lds_k : lds_acc;
  raise_lds_limits(sh, mlp_lds_bytes_eval(sh), lds);
  DPPO_DISPATCH(grad_kernel, sh, dim3((unsigned)G), lds, s, k);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
