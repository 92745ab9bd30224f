// Fused PPO minibatch step (gather -> forward -> loss -> analytic backward -> weight-gradient
// partials) on gfx950 fp32 MFMA, feature-split ("cooperative") form.
//
// Reference: loss and backward of one minibatch, diamond/ppo.py:261-283 (continuous:
// continuous_ppo.py:273-295), default networks ppo.py:53-71 / continuous_ppo.py:63-81.
//
// ---- Decomposition ----------------------------------------------------------------------------
// A workgroup = one team of 4 waves (256 threads, one workgroup per CU) processing 64 samples
// per step.  Every hidden layer (64 features) is split by OUTPUT feature across the team: wave q
// owns features [16q, 16q+16) of every layer, for every sample of the step.  So per wave:
//   * forward  Y[16q.., s] = W[16q.., :] X[:, s]      A = its 16-row slice of W (registers),
//   * backward dX[16q.., s] = W[:, 16q..]^T dZ[:, s]  A = its 16-column slice of W (registers),
//   * dW[16q.., :] += dZ[16q.., s] X[:, s]^T          accumulator: 16 rows x 64 = 16 registers,
// with v_mfma_f32_16x16x4_f32 (exact fp32).  Activations and deltas travel between waves
// through per-team LDS images [sample][feature]; a workgroup barrier separates the layer phases.
// The weight-gradient state per wave is 56 registers instead of 224 and each wave keeps its 104
// weight-slice registers resident; four independent 16-sample MFMA chains per wave hide the
// 16x16x4 MFMA latency.  The feature columns of every activation image are permuted inside each
// 16-column block, col(k) = 16(k>>4) + 4(k&3) + ((k>>2)&3), so that the 4 consecutive k-steps a
// lane feeds the MFMA B operand are 16 contiguous bytes (one ds_read_b128 per 4 MFMAs).
//
// Heads (logits / Gaussian mean, value) and the per-sample loss run on VALU: 8 lanes per sample.
// Head weight gradients are per-lane (lane = feature column) sums over samples.  Every
// accumulator is reduced in a fixed order at the end and written as ONE slab per workgroup
// (optim.hip sums the slabs in a fixed order): bit-reproducible, no float atomics.
#include "common.h"

namespace dppo {
namespace {

constexpr int H = 64;
constexpr int kTeamWaves = 4;
constexpr int kTeams = 1;
constexpr int kThreads = kTeams * kTeamWaves * kWave;  // 256
constexpr int S = 64;                                   // samples per team step
constexpr int NSB = S / 16;                             // 16-sample MFMA tiles per step
constexpr int SA = 68;                                  // stride of 64-col images
constexpr int SAC = 132;                                // stride of the [ha | hc] images
constexpr int SD = 68;                                  // stride of the per-sample head image
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
constexpr float kHalfLog2PiPlusHalf = 1.41893853320467274178f;

// Timing-only ablation switches (tools/ablate.py); a shipped build defines none of them.
#ifdef DPPO_ABL_NOBARRIER
#define STEP_BARRIER() __builtin_amdgcn_wave_barrier()
#else
#define STEP_BARRIER() __syncthreads()
#endif

__host__ __device__ constexpr int perm(int k) { return (k & ~15) + 4 * (k & 3) + ((k >> 2) & 3); }

struct TeamLds {  // offsets (floats) of one team's images
  int X0, H1, H2, HAC, DZAC, DOUT, DZ2;
  int size;
};

struct Lds2 {
  int Wo;  // [16][64] head weights, permuted columns
  int Wv;  // [64] permuted
  int b1, b2, ba, bc;  // [64] natural order
  int bo, ls, bv;      // [16] [16] [4]
  int team0;           // team images
  TeamLds t;
  int SX0;             // X0 stride
  int total;
};

struct MArgs {
  Lds2 L;
  ParamOffsets po;
  const float* params;
  const float* rec;
  const int32_t* idx;
  int m;
  float inv_m, clip_eps, vf, ent;
  float* slabs;
  int64_t slab_stride, p_total;
  int D, D8, D16, A, R;
};

inline int a4(int x) { return (x + 3) & ~3; }

Lds2 make_lds2(int D16) {
  Lds2 L{};
  int o = 0;
  L.Wo = o; o += 16 * H;
  L.Wv = o; o += H;
  L.b1 = o; o += H;
  L.b2 = o; o += H;
  L.ba = o; o += H;
  L.bc = o; o += H;
  L.bo = o; o += 16;
  L.ls = o; o += 16;
  L.bv = o; o += 4;
  L.team0 = o;
  L.SX0 = D16 + 4;
  TeamLds t{};
  int u = 0;
  t.X0 = u; u += a4(S * L.SX0);
  t.H1 = u; u += S * SA;
  t.H2 = u; u += S * SA;
  t.HAC = u; u += S * SAC;
  t.DZAC = u; u += S * SAC;
  t.DOUT = u; u += S * SD;
  t.DZ2 = u; u += S * SA;
  t.size = u;
  L.t = t;
  o += kTeams * u;
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

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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

// One 16-row output slice for 2 sample tiles: acc[sb] += W(regs, k = 4t + h4) x X(LDS image).
template <int NT>
__device__ __forceinline__ void mm_rows(f32x4 (&acc)[NSB], const float (&w)[NT], const float* X,
                                        int stride, int l15, int h4) {
#ifdef DPPO_ABL_NOMM
  return;
#endif
#pragma unroll
  for (int q = 0; q < NT / 4; ++q) {
    f32x4 b[NSB];
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb)
      b[sb] = *(const f32x4*)(X + (16 * sb + l15) * stride + 16 * q + 4 * h4);
    // consecutive MFMAs hit different accumulators (16x16x4 f32: 32-cycle issue, 40-cycle
    // dependent latency)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) acc[sb] = mfma16(w[4 * q + j], b[sb][j], acc[sb]);
  }
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
    for (int r = 0; r < 4; ++r) v[sb][r] = tanh_f(v[sb][r]);
}

// dW rows (16q..) += sum over the 32 staged samples: A = dZ image (cols perm(o)), B = X image.
template <int NIB>
__device__ __forceinline__ void wgrad16(f32x4* acc, const float* DZ, int dz_stride,
                                        int dz_col0, const float* X, int x_stride, int x_col0,
                                        int row0, int l15, int h4) {
#ifdef DPPO_ABL_NOWGRAD
  return;
#endif
  const int ca = dz_col0 + perm(row0 + l15);
#pragma unroll
  for (int t = 0; t < S / 4; ++t) {
    const int s = 4 * t + h4;
    const float a = DZ[s * dz_stride + ca];
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib) {
      const float b = X[s * x_stride + x_col0 + perm(16 * ib + l15)];
      acc[ib] = mfma16(a, b, acc[ib]);
    }
  }
}

template <int AMAX, bool CONT>
__global__ __launch_bounds__(kThreads, 1) void mb_kernel(MArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  float* lds = lds_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = wave;  // feature quarter owned by this wave
  const int l15 = lane & 15, h4 = lane >> 4;
  const Lds2& L = a.L;
  const float* P = a.params;
  const ParamOffsets& po = a.po;
  const int row0 = 16 * q;  // this wave's feature rows

  // ---------------- prologue: LDS head weights / biases, register weight slices
  for (int k = tid; k < 16 * H; k += kThreads) {
    const int r = k >> 6, f = k & 63;
    lds[L.Wo + r * H + perm(f)] = r < a.A ? P[po.Wo + r * H + f] : 0.0f;
  }
  for (int k = tid; k < H; k += kThreads) {
    lds[L.Wv + perm(k)] = P[po.Wv + k];
    lds[L.b1 + k] = P[po.b1 + k];
    lds[L.b2 + k] = P[po.b2 + k];
    lds[L.ba + k] = P[po.ba + k];
    lds[L.bc + k] = P[po.bc + k];
  }
  for (int k = tid; k < 16; k += kThreads) {
    lds[L.bo + k] = k < a.A ? P[po.bo + k] : 0.0f;
    lds[L.ls + k] = (po.ls >= 0 && k < a.A) ? P[po.ls + k] : 0.0f;
  }
  if (tid < 4) lds[L.bv + tid] = tid == 0 ? P[po.bv] : 0.0f;

  float w1f[8], w2f[16], waf[16], wcf[16], w2b[16], wab[16], wcb[16];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int k = 4 * t + h4;
    w1f[t] = k < a.D ? P[po.W1 + (row0 + l15) * a.D + k] : 0.0f;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int k = 4 * t + h4;
    w2f[t] = P[po.W2 + (row0 + l15) * H + k];
    waf[t] = P[po.Wa + (row0 + l15) * H + k];
    wcf[t] = P[po.Wc + (row0 + l15) * H + k];
    w2b[t] = P[po.W2 + k * H + row0 + l15];
    wab[t] = P[po.Wa + k * H + row0 + l15];
    wcb[t] = P[po.Wc + k * H + row0 + l15];
  }
  __syncthreads();

  const int SX0 = L.SX0;

  f32x4 gW1[2], gW2[4], gWa[4], gWc[4], gb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    gW2[i] = gWa[i] = gWc[i] = gb[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (i < 2) gW1[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  float gWo[AMAX];
#pragma unroll
  for (int k = 0; k < AMAX; ++k) gWo[k] = 0.f;
  float gWv = 0.f, gbh = 0.f, s_pi = 0.f, s_v = 0.f, s_ent = 0.f;

  // Gather / head phases: 8 lanes per sample; each wave owns samples [16q, 16q+16) of the step,
  // two passes of 8.
  const int hj = lane & 7;
  const int nk1 = a.D16 / 4;  // layer-1 k-steps (4 or 8)

  const int nsteps = (a.m + S - 1) / S;
  // Sample-record prefetch, one step ahead in two stages so no phase waits on a dependent
  // global round trip: the indices of step+1 are loaded after phase 1, the record fields
  // (observation chunk, {action, old log-prob, advantage, return}, continuous actions) after
  // phase 5; phases 6-9 cover their latency.
  constexpr int NA4 = CONT ? (AMAX + 3) / 4 : 1;
  int nidx[2];
  f32x4 pobs[2], psc[2], pact[2][NA4];
  auto load_idx = [&](int st) {
#pragma unroll
    for (int pss = 0; pss < 2; ++pss) {
      const int si = st * S + 16 * q + 8 * pss + (lane >> 3);
      nidx[pss] = (st < nsteps && si < a.m) ? a.idx[si] : 0;
    }
  };
  auto load_rec = [&](int st) {
#pragma unroll
    for (int pss = 0; pss < 2; ++pss) {
      const int si = st * S + 16 * q + 8 * pss + (lane >> 3);
      const bool valid = st < nsteps && si < a.m;
      const float* rec = a.rec + (int64_t)nidx[pss] * a.R;
      pobs[pss] = (valid && hj < nk1 && 4 * hj < a.D8) ? *(const f32x4*)(rec + 4 * hj)
                                                       : (f32x4){0.f, 0.f, 0.f, 0.f};
      psc[pss] = *(const f32x4*)(rec + a.D8);
#pragma unroll
      for (int c = 0; c < NA4; ++c)
        pact[pss][c] = (CONT && 4 * c < a.A) ? *(const f32x4*)(rec + a.D8 + 4 + 4 * c)
                                             : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
  };
  load_idx(blockIdx.x);
  load_rec(blockIdx.x);
  for (int step = blockIdx.x; step < nsteps; step += gridDim.x) {
    lds = opaque_base(lds_);
    float* T = lds + L.team0;
    float* X0 = T + L.t.X0;
    float* H1 = T + L.t.H1;
    float* H2 = T + L.t.H2;
    float* HAC = T + L.t.HAC;
    float* DZAC = T + L.t.DZAC;
    float* DOUT = T + L.t.DOUT;
    float* DZ2 = T + L.t.DZ2;
    float* DZ1 = HAC;  // HAC is dead after the head phase
    // ---- (1) gather: obs -> X0 (permuted cols)
#pragma unroll
    for (int pss = 0; pss < 2; ++pss) {
      const int hs = 16 * q + 8 * pss + (lane >> 3);
      if (hj < nk1) {
        const int kb = 4 * hj;
#pragma unroll
        for (int j = 0; j < 4; ++j) X0[hs * SX0 + perm(kb + j)] = pobs[pss][j];
      }
    }
    load_idx(step + gridDim.x);
    STEP_BARRIER();

    // ---- (2) layer 1
    f32x4 h1r[NSB], h2r[NSB], har[NSB], hcr[NSB];
    init_bias(h1r, lds + L.b1, row0, h4);
    if (nk1 == 8) {
      mm_rows<8>(h1r, w1f, X0, SX0, l15, h4);
    } else {
      const float w1h[4] = {w1f[0], w1f[1], w1f[2], w1f[3]};
      mm_rows<4>(h1r, w1h, X0, SX0, l15, h4);
    }
    tanh_rows(h1r);
    put_rows(H1, SA, row0, h1r, l15, h4);
    STEP_BARRIER();

    // ---- (3) layer 2
    init_bias(h2r, lds + L.b2, row0, h4);
    mm_rows<16>(h2r, w2f, H1, SA, l15, h4);
    tanh_rows(h2r);
    put_rows(H2, SA, row0, h2r, l15, h4);
    STEP_BARRIER();

    // ---- (4) actor / critic hidden layers
    init_bias(har, lds + L.ba, row0, h4);
    init_bias(hcr, lds + L.bc, row0, h4);
    mm_rows<16>(har, waf, H2, SA, l15, h4);
    mm_rows<16>(hcr, wcf, H2, SA, l15, h4);
    tanh_rows(har);
    tanh_rows(hcr);
    put_rows(HAC, SAC, row0, har, l15, h4);
    put_rows(HAC, SAC, 64 + row0, hcr, l15, h4);
    STEP_BARRIER();

    // ---- (5) heads + loss (VALU, 8 lanes per sample)
#ifdef DPPO_ABL_NOHEADS
    if (step < 0)
#endif
#pragma unroll
    for (int pss = 0; pss < 2; ++pss) {
      const int hs = 16 * q + 8 * pss + (lane >> 3);
      const int si = step * S + hs;
      const bool valid = si < a.m;
      const f32x4 sc = psc[pss];  // {action bits, old logp, adv, return}
      const float* hrow = HAC + hs * SAC;
      float out[AMAX];
#pragma unroll
      for (int k = 0; k < AMAX; ++k) {
        float part = 0.f;
        if (k < a.A) {
#pragma unroll
          for (int m8 = 0; m8 < 8; ++m8)
            part += lds[L.Wo + k * H + 8 * m8 + hj] * hrow[8 * m8 + hj];
        }
        part += __shfl_xor(part, 1);
        part += __shfl_xor(part, 2);
        part += __shfl_xor(part, 4);
        out[k] = part + lds[L.bo + k];
      }
      float vp = 0.f;
#pragma unroll
      for (int m8 = 0; m8 < 8; ++m8) vp += lds[L.Wv + 8 * m8 + hj] * hrow[64 + 8 * m8 + hj];
      vp += __shfl_xor(vp, 1);
      vp += __shfl_xor(vp, 2);
      vp += __shfl_xor(vp, 4);
      const float v = vp + lds[L.bv];
      const float adv = sc[2], ret = sc[3];
      float logp = 0.f, ent = 0.f;
      float p[AMAX], lp[AMAX], xa[AMAX], sig[AMAX];
      if (CONT) {
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
          xa[k] = 0.f;
          sig[k] = 1.f;
          if (k < a.A) {
            xa[k] = pact[pss][k >> 2][k & 3];
            sig[k] = __expf(lds[L.ls + k]);
            const float lsc = __logf(sig[k]);
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
          if (k < a.A) se += __expf(out[k] - mx);
        const float lse = mx + __logf(se);
#pragma unroll
        for (int k = 0; k < AMAX; ++k) {
          lp[k] = 0.f;
          p[k] = 0.f;
          if (k < a.A) {
            lp[k] = out[k] - lse;
            p[k] = __expf(lp[k]);
            ent -= p[k] * lp[k];
            if (k == act) logp = lp[k];
          }
        }
      }
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
        if (k < a.A && (k & 7) == hj) {
          float dk, dl = 0.f;
          if (CONT) {
            const float dd = xa[k] - out[k];
            const float z = dd / sig[k];
            dk = dlogp * dd / (sig[k] * sig[k]);
            dl = dlogp * (z * z - 1.0f);
          } else {
            const int act = __float_as_int(sc[0]);
            dk = dlogp * ((k == act ? 1.f : 0.f) - p[k]) + a.ent * vm * p[k] * (lp[k] + ent);
          }
          drow[k] = dk;
          if (CONT) drow[33 + k] = dl;
        }
      }
      if (hj == 0) drow[32] = dv;
    }
    load_rec(step + gridDim.x);
    STEP_BARRIER();

    // ---- (6) head weight gradients (lane = feature column) and dZa, dZc of this wave's rows
    {
#pragma unroll 2
      for (int j = 0; j < 16; ++j) {
        const int s = 16 * q + j;
        const float* drow = DOUT + s * SD;
        const float ha = HAC[s * SAC + lane];
        const float hc = HAC[s * SAC + 64 + lane];
#pragma unroll
        for (int k = 0; k < AMAX; ++k)
          if (k < a.A) gWo[k] += drow[k] * ha;
        gWv += drow[32] * hc;
        gbh += drow[lane];  // lanes < A: bo; lane 32: bv; lanes 33..: log-std terms
      }
      f32x4 dza[NSB], dzc[NSB];
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) {
        const float* drow = DOUT + (16 * sb + l15) * SD;
        const float dvs = drow[32];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int col = row0 + 4 * r + h4;  // perm(row0 + 4 h4 + r)
          float acc = 0.f;
#pragma unroll
          for (int k = 0; k < AMAX; ++k)
            if (k < a.A) acc += lds[L.Wo + k * H + col] * drow[k];
          const float y = har[sb][r];
          dza[sb][r] = acc * (1.0f - y * y);
          const float yc = hcr[sb][r];
          dzc[sb][r] = lds[L.Wv + col] * dvs * (1.0f - yc * yc);
        }
        gb[2] += dza[sb];
        gb[3] += dzc[sb];
      }
      put_rows(DZAC, SAC, row0, dza, l15, h4);
      put_rows(DZAC, SAC, 64 + row0, dzc, l15, h4);
    }
    STEP_BARRIER();

    // ---- (7) dh2 = Wa^T dZa + Wc^T dZc ; dZ2 ; dWa, dWc of this wave's rows
    {
      f32x4 dz2[NSB];
      zero(dz2);
      mm_rows<16>(dz2, wab, DZAC, SAC, l15, h4);
      mm_rows<16>(dz2, wcb, DZAC + 64, SAC, l15, h4);
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) dz2[sb][r] *= (1.0f - h2r[sb][r] * h2r[sb][r]);
        gb[1] += dz2[sb];
      }
      put_rows(DZ2, SA, row0, dz2, l15, h4);
      wgrad16<4>(gWa, DZAC, SAC, 0, H2, SA, 0, row0, l15, h4);
      wgrad16<4>(gWc, DZAC, SAC, 64, H2, SA, 0, row0, l15, h4);
    }
    STEP_BARRIER();

    // ---- (8) dh1 = W2^T dZ2 ; dZ1 ; dW2 of this wave's rows
    {
      f32x4 dz1[NSB];
      zero(dz1);
      mm_rows<16>(dz1, w2b, DZ2, SA, l15, h4);
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) dz1[sb][r] *= (1.0f - h1r[sb][r] * h1r[sb][r]);
        gb[0] += dz1[sb];
      }
      put_rows(DZ1, SA, row0, dz1, l15, h4);
      wgrad16<4>(gW2, DZ2, SA, 0, H1, SA, 0, row0, l15, h4);
    }
    STEP_BARRIER();

    // ---- (9) dW1 of this wave's rows (input = observations)
    if (nk1 == 8) wgrad16<2>(gW1, DZ1, SA, 0, X0, SX0, 0, row0, l15, h4);
    else wgrad16<1>(gW1, DZ1, SA, 0, X0, SX0, 0, row0, l15, h4);
    STEP_BARRIER();
  }

  // ---------------- epilogue -> one slab per workgroup.  Each wave owns distinct rows of dW1,
  // dW2, dWa, dWc and of the hidden biases, so it stores them straight to the slab (no cross-wave
  // sum).  Only the head partials (lane = feature column, summed over this wave's samples) and
  // the loss sums are combined across the 4 waves, through LDS in a fixed order.  Padding floats
  // of the flat layout are never written (the slabs were zeroed at dppo_create).
  float* slab = a.slabs + (int64_t)blockIdx.x * a.slab_stride;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = gb[i][r];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      gb[i][r] = v;
    }
  for (int off = 32; off >= 1; off >>= 1) {
    s_pi += __shfl_xor(s_pi, off);
    s_v += __shfl_xor(s_v, off);
    s_ent += __shfl_xor(s_ent, off);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int o = row0 + 4 * h4 + r;
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
      const int i = 16 * ib + l15;
      slab[po.W2 + o * H + i] = gW2[ib][r];
      slab[po.Wa + o * H + i] = gWa[ib][r];
      slab[po.Wc + o * H + i] = gWc[ib][r];
    }
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int i = 16 * ib + l15;
      if (i < a.D) slab[po.W1 + o * a.D + i] = gW1[ib][r];
    }
    if (l15 == 0) {
      slab[po.b1 + o] = gb[0][r];
      slab[po.b2 + o] = gb[1][r];
      slab[po.ba + o] = gb[2][r];
      slab[po.bc + o] = gb[3][r];
    }
  }
  // head partials: [wave][AMAX + 2 (Wv, bias/log-std column sums) + 1 (loss)][64] in LDS
  constexpr int NH = AMAX + 3;
  __syncthreads();  // all waves are done with the step images
  float* hp = lds_ + wave * NH * 64;
#pragma unroll
  for (int k = 0; k < AMAX; ++k) hp[k * 64 + lane] = gWo[k];
  hp[AMAX * 64 + lane] = gWv;
  hp[(AMAX + 1) * 64 + lane] = gbh;
  hp[(AMAX + 2) * 64 + lane] = lane == 0 ? s_pi : (lane == 1 ? s_v : (lane == 2 ? s_ent : 0.f));
  __syncthreads();
  const int fcol = lane;  // permuted feature column held by this lane
  const int c15 = fcol & 15;
  const int ftrue = (fcol & ~15) + 4 * (c15 & 3) + (c15 >> 2);
  for (int e = wave; e < NH; e += kThreads / 64) {
    const float v = ((lds_[0 * NH * 64 + e * 64 + lane] + lds_[1 * NH * 64 + e * 64 + lane]) +
                     lds_[2 * NH * 64 + e * 64 + lane]) + lds_[3 * NH * 64 + e * 64 + lane];
    if (e < AMAX) {
      if (e < a.A) slab[po.Wo + e * H + ftrue] = v;
    } else if (e == AMAX) {
      slab[po.Wv + ftrue] = v;
    } else if (e == AMAX + 1) {
      if (lane < a.A) slab[po.bo + lane] = v;
      if (lane == 32) slab[po.bv] = v;
      if (CONT && lane >= 33 && lane < 33 + a.A) slab[po.ls + (lane - 33)] = v;
    } else {
      if (lane < 3) slab[a.p_total + lane] = v;
    }
  }
}

}  // namespace

size_t mb_lds_bytes(const MlpShape& sh) {
  const int D16 = (sh.D + 15) / 16 * 16;
  return (size_t)make_lds2(D16).total * sizeof(float);
}

int mb_grid(int32_t m) {
  const int nsteps = (m + S - 1) / S;
  int g = nsteps;
  if (g > 256) g = 256;
  if (g < 1) g = 1;
  return g;
}

int launch_mb(const MlpShape& sh, const ParamOffsets& po, const GradArgs& ga, int G,
              hipStream_t s) {
  MArgs k{};
  const int D16 = (sh.D + 15) / 16 * 16;
  k.L = make_lds2(D16);
  k.po = po;
  k.params = ga.params;
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
  k.D = sh.D;
  k.D8 = sh.D8;
  k.D16 = D16;
  k.A = sh.A;
  k.R = sh.R;
  size_t lds = (size_t)k.L.total * sizeof(float);
  const size_t acc = (size_t)(ga.p_total + 8) * sizeof(float);
  if (acc > lds) lds = acc;
  static bool attr = false;
  if (!attr) {
    attr = true;
#define DPPO_SET2(A, C)                                                                       \
  (void)hipFuncSetAttribute((const void*)mb_kernel<A, C>,                                     \
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    DPPO_SET2(2, false) DPPO_SET2(2, true) DPPO_SET2(4, false) DPPO_SET2(4, true)
    DPPO_SET2(8, false) DPPO_SET2(8, true) DPPO_SET2(16, false) DPPO_SET2(16, true)
#undef DPPO_SET2
  }
  const dim3 grid((unsigned)G), block(kThreads);
  const bool c = sh.continuous != 0;
  if (sh.A <= 2) {
    if (c) hipLaunchKernelGGL((mb_kernel<2, true>), grid, block, lds, s, k);
    else hipLaunchKernelGGL((mb_kernel<2, false>), grid, block, lds, s, k);
  } else if (sh.A <= 4) {
    if (c) hipLaunchKernelGGL((mb_kernel<4, true>), grid, block, lds, s, k);
    else hipLaunchKernelGGL((mb_kernel<4, false>), grid, block, lds, s, k);
  } else if (sh.A <= 8) {
    if (c) hipLaunchKernelGGL((mb_kernel<8, true>), grid, block, lds, s, k);
    else hipLaunchKernelGGL((mb_kernel<8, false>), grid, block, lds, s, k);
  } else {
    if (c) hipLaunchKernelGGL((mb_kernel<16, true>), grid, block, lds, s, k);
    else hipLaunchKernelGGL((mb_kernel<16, false>), grid, block, lds, s, k);
  }
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
