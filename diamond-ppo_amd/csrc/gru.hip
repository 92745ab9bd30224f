// RecurrentPPO minibatch gradient, fused: the full [T x N] GRU sequence recomputed from the stored
// initial hidden state (intended semantics of reference diamond/recurrent_ppo.py:301-367: every
// minibatch re-runs the sequence, :337, and slices its samples, :340-341), the PPO loss on the
// minibatch's samples, and the analytic backward through heads, GRU (BPTT with the per-step hidden
// resets, :82-87) and base layer -- one launch per minibatch instead of torch's hundreds.  The
// reference itself cannot run (GRUCore.forward evaluates `hx or ...` on a tensor, :78), so the
// yardstick is torch's own nn.GRU cell on the same semantics (tests/test_gpu_gru.py).
//
// Network (recurrent_ppo.py:94-149 as restated in diamond/recurrent_ppo.py): x1 = tanh(Wb obs + bb)
// [64]; torch GRU cell, hidden G = 16: r = s(Wir x1 + bir + Whr h + bhr), z = s(Wiz x1 + biz + Whz h +
// bhz), n = tanh(Win x1 + bin + r (Whn h + bhn)), h' = (1 - z) n + z h, with h zeroed where the
// step's prev_done is set; actor Linear(16, 64) tanh Linear(64, A); critic Linear(16, 64) tanh
// Linear(64, 1).
//
// One workgroup = 16 envs over all T steps (256 threads).  Phases, separated by workgroup
// barriers, exchanging per-sample vectors through a global scratch (SoA, one row per sample):
//  A  per sample: x1 and the input half of the gates gi = Wih x1 + bih (VALU, weights in LDS);
//  B  per env, serial in t: 16 lanes per env (lane j = hidden unit j), the recurrent half
//     gh = Whh h + bhh and the cell; h exchanged through LDS inside the wave each step;
//  C  per minibatch sample: heads, loss (ppo.py:264-280 terms), head backward -> dL/dh';
//  D  per env, serial in reverse: BPTT through the cell -> dgi, dgh per step;
//  E  per sample: dx1 = (Wih^T dgi)(1 - x1^2);
//  F  weight gradients = sums over the workgroup's samples of outer products, on MFMA
//     (v_mfma_f32_16x16x4_f32, k = sample) in a fixed order; bias sums on VALU; one slab per
//     workgroup (optim.hip's slab reduction sums them in a fixed order: bit-reproducible).
#include <cstring>

#include "common.h"

namespace dppo {
namespace {

constexpr int kG = 16;        // GRU hidden
constexpr int kH = 64;        // MLP hidden
constexpr int kEnvs = 16;     // envs per workgroup
constexpr int kThr = 256;
constexpr int kAPad = 16;     // action dims padded

struct GruArgs {
  GruOffsets po;
  const float* params;
  dppo_gru_batch b;
  const float* wmask;  // [B] 1 for the minibatch's samples, else 0
  int T, N, D, D16, A;
  float inv_m, clip_eps, vf, ent;
  GruScratch sc;
  float* slabs;
  int64_t slab_stride, p_total;
};

// LDS image of the weights (floats)
struct GruLds {
  int Wb, bb, Wih, bih, Whh, bhh, Wa1, ba1, Wa2, ba2, Wc1, bc1, Wc2, bc2, hbuf, gbuf, red, total;
};
__host__ __device__ constexpr GruLds gru_lds(int D) {
  GruLds L{};
  int o = 0;
  L.Wb = o; o += kH * D;
  L.bb = o; o += kH;
  L.Wih = o; o += 3 * kG * kH;
  L.bih = o; o += 3 * kG;
  L.Whh = o; o += 3 * kG * kG;
  L.bhh = o; o += 3 * kG;
  L.Wa1 = o; o += kH * kG;
  L.ba1 = o; o += kH;
  L.Wa2 = o; o += kAPad * kH;
  L.ba2 = o; o += kAPad;
  L.Wc1 = o; o += kH * kG;
  L.bc1 = o; o += kH;
  L.Wc2 = o; o += kH;
  L.bc2 = o; o += 4;
  o = (o + 3) & ~3;
  L.hbuf = o; o += kEnvs * kG;
  L.gbuf = o; o += kEnvs * 3 * kG;
  L.red = o; o += 4 * kThr;
  L.total = o;
  return L;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_acc(float x) {
  // 1 - 2 / (e^{2x} + 1): saturates cleanly, ~1e-7 absolute
  return 1.0f - 2.0f / (__expf(2.0f * x) + 1.0f);
}

// Sum over k = samples of A[s][m] B[s][n] for one 16 x 16 output tile: rows mt*16.., cols nt*16..
// of arrays with row strides lda / ldb (floats).  Lane (q, r) supplies A[s_{4kk+q}][16mt + r] and
// B[s_{4kk+q}][16nt + r]; the result D[4q + v][r] lands in register v.  s_k enumerates the
// workgroup's samples (t, e) as t * N + n0 + e, e < ne, in t-major order.
__device__ __forceinline__ f32x4 tile_sum(const float* __restrict__ A, int lda, int mt,
                                          const float* __restrict__ B, int ldb, int nt, int S,
                                          int ne, int N, int n0, int q, int r) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < S; k0 += 4) {
    const int s = k0 + q;
    const bool ok = s < S;
    const int ss = ok ? s : S - 1;
    const int t = ss / ne, e = ss - t * ne;
    const int64_t i = (int64_t)t * N + n0 + e;
    const float a = ok ? A[i * lda + 16 * mt + r] : 0.0f;
    const float b = B[i * ldb + 16 * nt + r];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  return acc;
}

__global__ __launch_bounds__(kThr) void gru_grad_kernel(GruArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const GruLds L = gru_lds(a.D);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * kEnvs;
  const int ne = min(kEnvs, a.N - n0);
  const int T = a.T, N = a.N, D = a.D, A = a.A;
  const int S = T * ne;
  const float* P = a.params;
  const GruOffsets& po = a.po;
  const GruScratch& sc = a.sc;

  // ---- weights into LDS (Wa2 rows >= A and the pads zero)
  for (int k = tid; k < kH * D; k += kThr) lds[L.Wb + k] = P[po.Wb + k];
  for (int k = tid; k < 3 * kG * kH; k += kThr) lds[L.Wih + k] = P[po.Wih + k];
  for (int k = tid; k < 3 * kG * kG; k += kThr) lds[L.Whh + k] = P[po.Whh + k];
  for (int k = tid; k < kH * kG; k += kThr) {
    lds[L.Wa1 + k] = P[po.Wa1 + k];
    lds[L.Wc1 + k] = P[po.Wc1 + k];
  }
  for (int k = tid; k < kAPad * kH; k += kThr) lds[L.Wa2 + k] = (k >> 6) < A ? P[po.Wa2 + k] : 0.f;
  if (tid < kH) {
    lds[L.bb + tid] = P[po.bb + tid];
    lds[L.ba1 + tid] = P[po.ba1 + tid];
    lds[L.bc1 + tid] = P[po.bc1 + tid];
    lds[L.Wc2 + tid] = P[po.Wc2 + tid];
  }
  if (tid < 3 * kG) {
    lds[L.bih + tid] = P[po.bih + tid];
    lds[L.bhh + tid] = P[po.bhh + tid];
  }
  if (tid < kAPad) lds[L.ba2 + tid] = tid < A ? P[po.ba2 + tid] : 0.f;
  if (tid == 0) lds[L.bc2] = P[po.bc2];
  __syncthreads();

  // ---- A: x1 and gi per sample (thread per sample).  x1 is produced 8 features at a time,
  // stored and folded into the 48 gate accumulators at once: no per-thread array is ever
  // indexed by a run-time value (that would put it in scratch memory).
  for (int s = tid; s < S; s += kThr) {
    const int t = s / ne, e = s - t * ne;
    const int64_t i = (int64_t)t * N + n0 + e;
    float ob[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) ob[c] = c < D ? a.b.obs[i * D + c] : 0.f;
    float* ob16 = sc.obs + i * a.D16;
#pragma unroll
    for (int c = 0; c < 32; ++c)
      if (c < a.D16) ob16[c] = ob[c];
    float gi[3 * kG];
#pragma unroll
    for (int g = 0; g < 3 * kG; ++g) gi[g] = lds[L.bih + g];
#pragma unroll 1
    for (int o0 = 0; o0 < kH; o0 += 8) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float z = lds[L.bb + o0 + u];
#pragma unroll
        for (int c = 0; c < 32; ++c)
          if (c < D) z += lds[L.Wb + (o0 + u) * D + c] * ob[c];
        x[u] = tanh_acc(z);
      }
      f32x4* xo = (f32x4*)(sc.x1 + i * kH + o0);
      xo[0] = (f32x4){x[0], x[1], x[2], x[3]};
      xo[1] = (f32x4){x[4], x[5], x[6], x[7]};
#pragma unroll
      for (int g = 0; g < 3 * kG; ++g) {
        const f32x4 w0 = *(const f32x4*)(lds + L.Wih + g * kH + o0);
        const f32x4 w1 = *(const f32x4*)(lds + L.Wih + g * kH + o0 + 4);
        gi[g] += ((w0[0] * x[0] + w0[1] * x[1]) + (w0[2] * x[2] + w0[3] * x[3])) +
                 ((w1[0] * x[4] + w1[1] * x[5]) + (w1[2] * x[6] + w1[3] * x[7]));
      }
    }
    f32x4* go = (f32x4*)(sc.gi + i * 3 * kG);
#pragma unroll
    for (int g = 0; g < 3 * kG / 4; ++g)
      go[g] = (f32x4){gi[4 * g], gi[4 * g + 1], gi[4 * g + 2], gi[4 * g + 3]};
  }
  __syncthreads();

  // ---- B: forward recurrence, lane j of env e = hidden unit j (16 lanes of one wave per env)
  const int e = tid >> 4, j = tid & 15;
  const bool env_ok = e < ne;
  const int n = n0 + e;
  if (env_ok) {
    float wr[kG], wz[kG], wn[kG];
#pragma unroll
    for (int k = 0; k < kG; ++k) {
      wr[k] = lds[L.Whh + j * kG + k];
      wz[k] = lds[L.Whh + (kG + j) * kG + k];
      wn[k] = lds[L.Whh + (2 * kG + j) * kG + k];
    }
    const float br = lds[L.bhh + j], bz = lds[L.bhh + kG + j], bn = lds[L.bhh + 2 * kG + j];
    float h = a.b.hx0[(int64_t)n * kG + j];
    float* hb = lds + L.hbuf + e * kG;
    for (int t = 0; t < T; ++t) {
      const int64_t i = (int64_t)t * N + n;
      if (a.b.prev_dones[i]) h = 0.0f;  // hx[:, dones[t]] = 0 (recurrent_ppo.py:84)
      hb[j] = h;
      const float gir = sc.gi[i * 3 * kG + j], giz = sc.gi[i * 3 * kG + kG + j],
                  gin = sc.gi[i * 3 * kG + 2 * kG + j];
      float hv[kG];
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f32x4 x = *(const f32x4*)(hb + 4 * q);
        hv[4 * q] = x[0];
        hv[4 * q + 1] = x[1];
        hv[4 * q + 2] = x[2];
        hv[4 * q + 3] = x[3];
      }
      float ghr = br, ghz = bz, ghn = bn;
#pragma unroll
      for (int k = 0; k < kG; ++k) {
        ghr += wr[k] * hv[k];
        ghz += wz[k] * hv[k];
        ghn += wn[k] * hv[k];
      }
      const float r = sigm(gir + ghr), z = sigm(giz + ghz);
      const float nn = tanh_acc(gin + r * ghn);
      const float hn = (1.0f - z) * nn + z * h;
      sc.hi[i * kG + j] = h;
      sc.r[i * kG + j] = r;
      sc.z[i * kG + j] = z;
      sc.n[i * kG + j] = nn;
      sc.ghn[i * kG + j] = ghn;
      sc.ho[i * kG + j] = hn;
      h = hn;
    }
  }
  __syncthreads();

  // ---- C: heads, loss and head backward per sample (ppo.py:264-280 with the GRU features).
  // Forward 8 head features at a time (stored, and folded into the logits / value at once);
  // backward the same blocks re-read from the scratch rows this thread just wrote.
  float s_pi = 0.f, s_v = 0.f, s_ent = 0.f;
  for (int s = tid; s < S; s += kThr) {
    const int t = s / ne, ee = s - t * ne;
    const int64_t i = (int64_t)t * N + n0 + ee;
    const float w = a.wmask[i];
    float dho[kG], dl[kAPad];
    float dv = 0.f;
#pragma unroll
    for (int k = 0; k < kAPad; ++k) dl[k] = 0.f;
#pragma unroll
    for (int k = 0; k < kG; ++k) dho[k] = 0.f;
    float* yar = sc.ya + i * kH;
    float* ycr = sc.yc + i * kH;
    float* dyar = sc.dya + i * kH;
    float* dycr = sc.dyc + i * kH;
    if (w != 0.f) {
      float hv[kG];
#pragma unroll
      for (int q = 0; q < kG / 4; ++q) {
        const f32x4 x = ((const f32x4*)(sc.ho + i * kG))[q];
        hv[4 * q] = x[0];
        hv[4 * q + 1] = x[1];
        hv[4 * q + 2] = x[2];
        hv[4 * q + 3] = x[3];
      }
      float out[kAPad];
#pragma unroll
      for (int k = 0; k < kAPad; ++k) out[k] = lds[L.ba2 + k];
      float val = lds[L.bc2];
#pragma unroll 1
      for (int o0 = 0; o0 < kH; o0 += 8) {
        float ya[8], yc[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float za = lds[L.ba1 + o0 + u], zc = lds[L.bc1 + o0 + u];
#pragma unroll
          for (int q = 0; q < kG / 4; ++q) {
            const f32x4 wa = *(const f32x4*)(lds + L.Wa1 + (o0 + u) * kG + 4 * q);
            const f32x4 wc = *(const f32x4*)(lds + L.Wc1 + (o0 + u) * kG + 4 * q);
            za += (wa[0] * hv[4 * q] + wa[1] * hv[4 * q + 1]) + (wa[2] * hv[4 * q + 2] + wa[3] * hv[4 * q + 3]);
            zc += (wc[0] * hv[4 * q] + wc[1] * hv[4 * q + 1]) + (wc[2] * hv[4 * q + 2] + wc[3] * hv[4 * q + 3]);
          }
          ya[u] = tanh_acc(za);
          yc[u] = tanh_acc(zc);
        }
        ((f32x4*)(yar + o0))[0] = (f32x4){ya[0], ya[1], ya[2], ya[3]};
        ((f32x4*)(yar + o0))[1] = (f32x4){ya[4], ya[5], ya[6], ya[7]};
        ((f32x4*)(ycr + o0))[0] = (f32x4){yc[0], yc[1], yc[2], yc[3]};
        ((f32x4*)(ycr + o0))[1] = (f32x4){yc[4], yc[5], yc[6], yc[7]};
#pragma unroll
        for (int k = 0; k < kAPad; ++k) {
          if (k < A) {
            const f32x4 w0 = *(const f32x4*)(lds + L.Wa2 + k * kH + o0);
            const f32x4 w1 = *(const f32x4*)(lds + L.Wa2 + k * kH + o0 + 4);
            out[k] += ((w0[0] * ya[0] + w0[1] * ya[1]) + (w0[2] * ya[2] + w0[3] * ya[3])) +
                      ((w1[0] * ya[4] + w1[1] * ya[5]) + (w1[2] * ya[6] + w1[3] * ya[7]));
          }
        }
        const f32x4 v0 = *(const f32x4*)(lds + L.Wc2 + o0);
        const f32x4 v1 = *(const f32x4*)(lds + L.Wc2 + o0 + 4);
        val += ((v0[0] * yc[0] + v0[1] * yc[1]) + (v0[2] * yc[2] + v0[3] * yc[3])) +
               ((v1[0] * yc[4] + v1[1] * yc[5]) + (v1[2] * yc[6] + v1[3] * yc[7]));
      }
      const int act = a.b.actions[i];
      float mx = out[0];
#pragma unroll
      for (int k = 1; k < kAPad; ++k)
        if (k < A) mx = fmaxf(mx, out[k]);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < kAPad; ++k)
        if (k < A) se += __expf(out[k] - mx);
      const float lse = mx + __logf(se);
      float ent = 0.f, logp = 0.f;
#pragma unroll
      for (int k = 0; k < kAPad; ++k) {
        const float lpk = out[k] - lse;
        const float pk = k < A ? __expf(lpk) : 0.f;
        ent -= pk * lpk;
        logp = k == act ? lpk : logp;
        out[k] = lpk;  // log-probabilities from here on
      }
      const float adv = a.b.advantages[i], ret = a.b.returns[i];
      const float ratio = __expf(logp - a.b.old_log_probs[i]);                 // ppo.py:266
      const float rcl = fminf(fmaxf(ratio, 1.0f - a.clip_eps), 1.0f + a.clip_eps);
      const float u = -adv * ratio, wv = -adv * rcl;                            // ppo.py:267-269
      const float inr = (ratio >= 1.0f - a.clip_eps && ratio <= 1.0f + a.clip_eps) ? 1.f : 0.f;
      const float gu = u > wv ? 1.f : (u == wv ? 0.5f : 0.f);  // torch.max splits ties
      const float gw = wv > u ? 1.f : (u == wv ? 0.5f : 0.f);
      const float vm = w * a.inv_m;
      const float dlogp = (gu * -adv + gw * -adv * inr) * vm * ratio;
      dv = a.vf * (val - ret) * vm;                                            // ppo.py:272
      s_pi += fmaxf(u, wv);
      s_v += 0.5f * (val - ret) * (val - ret);
      s_ent += ent;
#pragma unroll
      for (int k = 0; k < kAPad; ++k) {
        const float pk = k < A ? __expf(out[k]) : 0.f;
        dl[k] = k < A ? dlogp * ((k == act ? 1.f : 0.f) - pk) + a.ent * vm * pk * (out[k] + ent)
                      : 0.f;
      }
      // head backward: dya = (Wa2^T dl)(1 - ya^2), dyc = Wc2 dv (1 - yc^2),
      // dh' = Wa1^T dya + Wc1^T dyc
#pragma unroll 1
      for (int o0 = 0; o0 < kH; o0 += 4) {
        const f32x4 ya = *(const f32x4*)(yar + o0);
        const f32x4 yc = *(const f32x4*)(ycr + o0);
        f32x4 da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < kAPad; ++k)
          if (k < A) da += *(const f32x4*)(lds + L.Wa2 + k * kH + o0) * dl[k];
        const f32x4 dya = da * (1.0f - ya * ya);
        const f32x4 dyc = *(const f32x4*)(lds + L.Wc2 + o0) * dv * (1.0f - yc * yc);
        *(f32x4*)(dyar + o0) = dya;
        *(f32x4*)(dycr + o0) = dyc;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int q = 0; q < kG / 4; ++q) {
            const f32x4 wa = *(const f32x4*)(lds + L.Wa1 + (o0 + u) * kG + 4 * q);
            const f32x4 wc = *(const f32x4*)(lds + L.Wc1 + (o0 + u) * kG + 4 * q);
#pragma unroll
            for (int x = 0; x < 4; ++x) dho[4 * q + x] += wa[x] * dya[u] + wc[x] * dyc[u];
          }
        }
      }
    } else {
      const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int o = 0; o < kH / 4; ++o) {
        ((f32x4*)yar)[o] = zero;
        ((f32x4*)ycr)[o] = zero;
        ((f32x4*)dyar)[o] = zero;
        ((f32x4*)dycr)[o] = zero;
      }
    }
#pragma unroll
    for (int k = 0; k < kG / 4; ++k)
      ((f32x4*)(sc.dho + i * kG))[k] = (f32x4){dho[4 * k], dho[4 * k + 1], dho[4 * k + 2], dho[4 * k + 3]};
#pragma unroll
    for (int k = 0; k < kAPad / 4; ++k)
      ((f32x4*)(sc.dl + i * kAPad))[k] = (f32x4){dl[4 * k], dl[4 * k + 1], dl[4 * k + 2], dl[4 * k + 3]};
    ((f32x4*)(sc.dv + i * kAPad))[0] = (f32x4){dv, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 1; k < kAPad / 4; ++k) ((f32x4*)(sc.dv + i * kAPad))[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();

  // ---- D: BPTT, reverse in t (lane j of env e)
  if (env_ok) {
    float wc[3 * kG];  // column j of Whh
#pragma unroll
    for (int g = 0; g < 3 * kG; ++g) wc[g] = lds[L.Whh + g * kG + j];
    float* gb = lds + L.gbuf + e * 3 * kG;
    float carry = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const int64_t i = (int64_t)t * N + n;
      const float dh = sc.dho[i * kG + j] + carry;
      const float z = sc.z[i * kG + j], nn = sc.n[i * kG + j], r = sc.r[i * kG + j];
      const float hin = sc.hi[i * kG + j], ghn = sc.ghn[i * kG + j];
      const float dn = dh * (1.0f - z);
      const float dz = dh * (hin - nn);
      const float dnp = dn * (1.0f - nn * nn);
      const float dghn = dnp * r;
      const float drp = dnp * ghn * r * (1.0f - r);
      const float dzp = dz * z * (1.0f - z);
      float* dgi = sc.dgi + i * 3 * kG;
      float* dgh = sc.dgh + i * 3 * kG;
      dgi[j] = drp;
      dgi[kG + j] = dzp;
      dgi[2 * kG + j] = dnp;
      dgh[j] = drp;
      dgh[kG + j] = dzp;
      dgh[2 * kG + j] = dghn;
      gb[j] = drp;
      gb[kG + j] = dzp;
      gb[2 * kG + j] = dghn;
      float dhin = dh * z;
#pragma unroll
      for (int q = 0; q < 3 * kG / 4; ++q) {
        const f32x4 x = *(const f32x4*)(gb + 4 * q);
        dhin += wc[4 * q] * x[0] + wc[4 * q + 1] * x[1] + wc[4 * q + 2] * x[2] + wc[4 * q + 3] * x[3];
      }
      // h_in = h_prev * keep  =>  dh_prev = dh_in * keep
      carry = a.b.prev_dones[i] ? 0.0f : dhin;
    }
  }
  __syncthreads();

  // ---- E: dx1 = (Wih^T dgi)(1 - x1^2) per sample, 4 features at a time
  for (int s = tid; s < S; s += kThr) {
    const int t = s / ne, ee = s - t * ne;
    const int64_t i = (int64_t)t * N + n0 + ee;
    float dg[3 * kG];
#pragma unroll
    for (int g = 0; g < 3 * kG / 4; ++g) {
      const f32x4 x = ((const f32x4*)(sc.dgi + i * 3 * kG))[g];
      dg[4 * g] = x[0];
      dg[4 * g + 1] = x[1];
      dg[4 * g + 2] = x[2];
      dg[4 * g + 3] = x[3];
    }
    const float* x1 = sc.x1 + i * kH;
    float* dx = sc.dx1 + i * kH;
#pragma unroll 1
    for (int c0 = 0; c0 < kH; c0 += 4) {
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 3 * kG; ++g) d += *(const f32x4*)(lds + L.Wih + g * kH + c0) * dg[g];
      const f32x4 x = *(const f32x4*)(x1 + c0);
      *(f32x4*)(dx + c0) = d * (1.0f - x * x);
    }
  }
  __syncthreads();

  // ---- F: weight gradients (MFMA over samples), biases and loss sums into this workgroup's slab
  float* slab = a.slabs + (int64_t)blockIdx.x * a.slab_stride;
  {
    const int q = lane >> 4, r = lane & 15;
    const int nD = a.D16 / 16;
    // tiles: Wb 4 x nD | Wih 3 x 4 | Whh 3 x 1 | Wa1 4 x 1 | Wc1 4 x 1 | Wa2 1 x 4 | Wc2 1 x 4
    const int nt_b = 4 * nD, nt_ih = 12, nt_hh = 3, nt_a1 = 4, nt_c1 = 4, nt_a2 = 4, nt_c2 = 4;
    const int ntiles = nt_b + nt_ih + nt_hh + nt_a1 + nt_c1 + nt_a2 + nt_c2;
    for (int tl = wave; tl < ntiles; tl += kThr / 64) {
      int k = tl;
      const float *Aa, *Bb;
      int lda, ldb, mt, nt, rows, cols, ldo;
      int64_t off;
      if (k < nt_b) {
        Aa = sc.dx1; lda = kH; Bb = sc.obs; ldb = a.D16; mt = k / nD; nt = k % nD;
        off = po.Wb; rows = kH; cols = D; ldo = D;
      } else if ((k -= nt_b) < nt_ih) {
        Aa = sc.dgi; lda = 3 * kG; Bb = sc.x1; ldb = kH; mt = k / 4; nt = k % 4;
        off = po.Wih; rows = 3 * kG; cols = kH; ldo = kH;
      } else if ((k -= nt_ih) < nt_hh) {
        Aa = sc.dgh; lda = 3 * kG; Bb = sc.hi; ldb = kG; mt = k; nt = 0;
        off = po.Whh; rows = 3 * kG; cols = kG; ldo = kG;
      } else if ((k -= nt_hh) < nt_a1) {
        Aa = sc.dya; lda = kH; Bb = sc.ho; ldb = kG; mt = k; nt = 0;
        off = po.Wa1; rows = kH; cols = kG; ldo = kG;
      } else if ((k -= nt_a1) < nt_c1) {
        Aa = sc.dyc; lda = kH; Bb = sc.ho; ldb = kG; mt = k; nt = 0;
        off = po.Wc1; rows = kH; cols = kG; ldo = kG;
      } else if ((k -= nt_c1) < nt_a2) {
        Aa = sc.dl; lda = kAPad; Bb = sc.ya; ldb = kH; mt = 0; nt = k;
        off = po.Wa2; rows = A; cols = kH; ldo = kH;
      } else {
        k -= nt_a2;
        Aa = sc.dv; lda = kAPad; Bb = sc.yc; ldb = kH; mt = 0; nt = k;
        off = po.Wc2; rows = 1; cols = kH; ldo = kH;
      }
      const f32x4 acc = tile_sum(Aa, lda, mt, Bb, ldb, nt, S, ne, N, n0, q, r);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = 16 * mt + 4 * q + v, col = 16 * nt + r;
        if (row < rows && col < cols) slab[off + (int64_t)row * ldo + col] = acc[v];
      }
    }
  }
  {
    // bias columns: bb 64 | bih 48 | bhh 48 | ba1 64 | bc1 64 | ba2 A | bc2 1
    const int nb = kH + 3 * kG + 3 * kG + kH + kH + A + 1;
    for (int c = tid; c < nb; c += kThr) {
      const float* src;
      int ld, col;
      int64_t off;
      int k = c;
      if (k < kH) { src = sc.dx1; ld = kH; col = k; off = po.bb + k; }
      else if ((k -= kH) < 3 * kG) { src = sc.dgi; ld = 3 * kG; col = k; off = po.bih + k; }
      else if ((k -= 3 * kG) < 3 * kG) { src = sc.dgh; ld = 3 * kG; col = k; off = po.bhh + k; }
      else if ((k -= 3 * kG) < kH) { src = sc.dya; ld = kH; col = k; off = po.ba1 + k; }
      else if ((k -= kH) < kH) { src = sc.dyc; ld = kH; col = k; off = po.bc1 + k; }
      else if ((k -= kH) < A) { src = sc.dl; ld = kAPad; col = k; off = po.ba2 + k; }
      else { src = sc.dv; ld = kAPad; col = 0; off = po.bc2; }
      float sum = 0.f;
      for (int s = 0; s < S; ++s) {
        const int t = s / ne, ee = s - t * ne;
        sum += src[((int64_t)t * N + n0 + ee) * ld + col];
      }
      slab[off] = sum;
    }
  }
  // loss sums {policy, value, entropy} in a fixed order
  float* red = lds + L.red;
  red[tid] = s_pi;
  red[kThr + tid] = s_v;
  red[2 * kThr + tid] = s_ent;
  __syncthreads();
  if (tid < 3) {
    float sum = 0.f;
    for (int k = 0; k < kThr; ++k) sum += red[tid * kThr + k];
    slab[a.p_total + tid] = sum;
  }
}

__global__ void mask_kernel(const int32_t* __restrict__ idx, int m, float* __restrict__ wmask) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x)
    wmask[idx[k]] = 1.0f;
}

}  // namespace

size_t gru_lds_bytes(int D) { return (size_t)gru_lds(D).total * sizeof(float); }

int launch_gru_grad(const GruOffsets& po, const float* params, const dppo_gru_batch& b,
                    const int32_t* idx, int32_t m, float* wmask, int64_t B, int T, int N, int D,
                    int A, float inv_m, float clip_eps, float vf, float ent, const GruScratch& sc,
                    float* slabs, int64_t slab_stride, int64_t p_total, hipStream_t s) {
  DPPO_HIP_CHECK(hipMemsetAsync(wmask, 0, (size_t)B * sizeof(float), s));
  if (m > 0) {
    int g = (m + 255) / 256;
    if (g > 1024) g = 1024;
    DPPO_LAUNCH(mask_kernel, dim3(g), dim3(256), 0, s, idx, m, wmask);
    DPPO_LAUNCH_CHECK();
  }
  GruArgs a{};
  a.po = po;
  a.params = params;
  a.b = b;
  a.wmask = wmask;
  a.T = T;
  a.N = N;
  a.D = D;
  a.D16 = (D + 15) / 16 * 16;
  a.A = A;
  a.inv_m = inv_m;
  a.clip_eps = clip_eps;
  a.vf = vf;
  a.ent = ent;
  a.sc = sc;
  a.slabs = slabs;
  a.slab_stride = slab_stride;
  a.p_total = p_total;
  const size_t lds = gru_lds_bytes(D);
  const int grid = (N + kEnvs - 1) / kEnvs;
  DPPO_LAUNCH(gru_grad_kernel, dim3(grid), dim3(kThr), lds, s, a);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int gru_grid(int N) { return (N + kEnvs - 1) / kEnvs; }

}  // namespace dppo

// ---------------------------------------------------------------------------------------------
// C ABI (include/dppo.h): handle = workspace for one rollout shape.
using namespace dppo;

struct dppo_gru_handle {
  int device = 0;
  dppo_gru_dims dims{};
  dppo_layout layout{};
  GruOffsets po{};
  int64_t B = 0;
  int G = 1;
  int64_t slab_stride = 0;
  float* scratch = nullptr;  // one allocation, carved into GruScratch
  GruScratch sc{};
  float* wmask = nullptr;
  float* slabs = nullptr;
  double* sq_part = nullptr;
};

namespace {

int gru_validate(const dppo_gru_dims* d) {
  if (!d || d->rollout_steps < 1 || d->num_envs < 1 || d->obs_dim < 1 || d->act_dim < 1) {
    set_error("invalid dppo_gru_dims");
    return DPPO_EINVAL;
  }
  if (d->hidden != kH || d->gru_hidden != kG || d->obs_dim > 32 || d->act_dim > kAPad) {
    set_error("fused GRU kernels support hidden=64, gru_hidden=16, obs_dim<=32, act_dim<=16 "
              "(got H=%d G=%d D=%d A=%d)", d->hidden, d->gru_hidden, d->obs_dim, d->act_dim);
    return DPPO_EUNSUPPORTED;
  }
  if ((int64_t)d->rollout_steps * d->num_envs > 0x7FFFFFFF / 64) {
    set_error("T*N too large for the GRU workspace");
    return DPPO_EINVAL;
  }
  return DPPO_OK;
}

void gru_layout(const dppo_gru_dims* d, dppo_layout* L) {
  std::memset(L, 0, sizeof(*L));
  const int D = d->obs_dim, A = d->act_dim;
  // RecurrentActorCriticNetwork.named_parameters() order (diamond/recurrent_ppo.py)
  const int rc[14][2] = {{kH, D}, {kH, 1}, {3 * kG, kH}, {3 * kG, kG}, {3 * kG, 1}, {3 * kG, 1},
                         {kH, kG}, {kH, 1}, {A, kH}, {A, 1}, {kH, kG}, {kH, 1}, {1, kH}, {1, 1}};
  int64_t off = 0, real = 0;
  for (int i = 0; i < 14; ++i) {
    const int64_t ne = (int64_t)rc[i][0] * rc[i][1];
    L->offset[i] = off;
    L->numel[i] = ne;
    L->rows[i] = rc[i][0];
    L->cols[i] = rc[i][1];
    off = (off + ne + 15) / 16 * 16;
    real += ne;
  }
  L->count = 14;
  L->total = off;
  L->n_real = real;
}

}  // namespace

extern "C" {

int dppo_gru_param_layout(const dppo_gru_dims* dims, dppo_layout* out) {
  if (!out) {
    set_error("out is NULL");
    return DPPO_EINVAL;
  }
  const int rc = gru_validate(dims);
  if (rc != DPPO_OK && rc != DPPO_EUNSUPPORTED) return rc;
  gru_layout(dims, out);
  return DPPO_OK;
}

void dppo_gru_destroy(dppo_gru_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  (void)hipFree(h->scratch);
  (void)hipFree(h->wmask);
  (void)hipFree(h->slabs);
  (void)hipFree(h->sq_part);
  delete h;
}

int dppo_gru_create(int device, const dppo_gru_dims* dims, dppo_gru_handle** out) {
  if (!out) {
    set_error("out is NULL");
    return DPPO_EINVAL;
  }
  *out = nullptr;
  const int rc = gru_validate(dims);
  if (rc != DPPO_OK) return rc;
  DPPO_HIP_CHECK(hipSetDevice(device));
  dppo_gru_handle* h = new dppo_gru_handle();
  h->device = device;
  h->dims = *dims;
  gru_layout(dims, &h->layout);
  const int64_t* o = h->layout.offset;
  h->po = GruOffsets{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8], o[9], o[10], o[11],
                     o[12], o[13]};
  h->B = (int64_t)dims->rollout_steps * dims->num_envs;
  h->G = gru_grid(dims->num_envs);
  h->slab_stride = (h->layout.total + 8 + 63) / 64 * 64;
  const int D16 = (dims->obs_dim + 15) / 16 * 16;
  // per-sample rows: obs D16 | x1 64 | gi 48 | hi ho r z n ghn 6x16 | ya yc 2x64 | dl dv 2x16 |
  // dya dyc 2x64 | dho 16 | dgi dgh 2x48 | dx1 64
  const int64_t row = D16 + kH + 3 * kG + 6 * kG + 2 * kH + 2 * kAPad + 2 * kH + kG + 6 * kG + kH;
  hipError_t e = hipMalloc((void**)&h->scratch, (size_t)(h->B * row) * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&h->wmask, (size_t)h->B * sizeof(float));
  if (e == hipSuccess) e = hipMalloc((void**)&h->slabs, (size_t)(h->G * h->slab_stride) * sizeof(float));
  if (e == hipSuccess)
    e = hipMalloc((void**)&h->sq_part, (size_t)slab_reduce_blocks(h->layout.total) * sizeof(double));
  if (e != hipSuccess) {
    set_error("hipMalloc (GRU workspace) failed: %s", hipGetErrorString(e));
    dppo_gru_destroy(h);
    return DPPO_ENOMEM;
  }
  // the kernel never writes the layout's padding floats or the unused loss slots
  (void)hipMemset(h->slabs, 0, (size_t)(h->G * h->slab_stride) * sizeof(float));
  float* p = h->scratch;
  auto take = [&](int64_t w) {
    float* q = p;
    p += h->B * w;
    return q;
  };
  GruScratch& sc = h->sc;
  sc.obs = take(D16);
  sc.x1 = take(kH);
  sc.gi = take(3 * kG);
  sc.hi = take(kG);
  sc.ho = take(kG);
  sc.r = take(kG);
  sc.z = take(kG);
  sc.n = take(kG);
  sc.ghn = take(kG);
  sc.ya = take(kH);
  sc.yc = take(kH);
  sc.dl = take(kAPad);
  sc.dv = take(kAPad);
  sc.dya = take(kH);
  sc.dyc = take(kH);
  sc.dho = take(kG);
  sc.dgi = take(3 * kG);
  sc.dgh = take(3 * kG);
  sc.dx1 = take(kH);
  *out = h;
  return DPPO_OK;
}

int dppo_gru_minibatch_grad_f32(dppo_gru_handle* h, const float* params,
                                const dppo_gru_batch* batch, const int32_t* idx, int32_t m,
                                int32_t m_total, const dppo_hparams* hp, float* grad,
                                void* stream) {
  if (!h || !params || !batch || !idx || !hp || !grad || m < 0 || m_total <= 0 ||
      m > h->B || !batch->obs || !batch->actions || !batch->old_log_probs || !batch->advantages ||
      !batch->returns || !batch->prev_dones || !batch->hx0) {
    set_error("invalid argument to dppo_gru_minibatch_grad_f32");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t s = (hipStream_t)stream;
  static const bool attr = [] {
    raise_dyn_lds((const void*)gru_grad_kernel);
    return true;
  }();
  (void)attr;
  const dppo_gru_dims& d = h->dims;
  int rc = launch_gru_grad(h->po, params, *batch, idx, m, h->wmask, h->B, d.rollout_steps,
                           d.num_envs, d.obs_dim, d.act_dim, (float)(1.0 / (double)m_total),
                           hp->ppo_clip, hp->value_loss_weight, hp->entropy_beta, h->sc, h->slabs,
                           h->slab_stride, h->layout.total, s);
  if (rc != DPPO_OK) return rc;
  return launch_slab_reduce(h->slabs, h->G, h->slab_stride, h->layout.total, grad, h->sq_part, -1,
                            0, 0.0f, 0, s);
}

}  // extern "C"
