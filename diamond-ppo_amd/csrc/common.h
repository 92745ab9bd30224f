// Device-side common definitions for the gfx950 kernels of libdppo.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dppo_host.h"

#define DPPO_HIP_CHECK(expr)                                                              \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      ::dppo::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,  \
                        __LINE__);                                                        \
      return DPPO_EHIP;                                                                   \
    }                                                                                     \
  } while (0)

// Raise a kernel's dynamic-LDS limit to what a CU has left beside the kernel's static LDS (a
// request past 160 KiB in total fails, and a failed hipFuncSetAttribute leaves its error for the
// next hipGetLastError -- i.e. the next launch check).  Callers run it once per process through a
// function-local static initialiser, so concurrent launching threads (loopback groups) all wait
// for it instead of racing past a half-set limit.
inline void raise_dyn_lds(const void* fn) {
  hipFuncAttributes at{};
  size_t stat = 0;
  if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(160 * 1024 - stat));
  (void)hipGetLastError();
}

#define DPPO_LAUNCH_CHECK()                                                               \
  do {                                                                                    \
    hipError_t e_ = hipGetLastError();                                                    \
    if (e_ != hipSuccess) {                                                               \
      ::dppo::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(e_),        \
                        __FILE__, __LINE__);                                              \
      return DPPO_EHIP;                                                                   \
    }                                                                                     \
  } while (0)

namespace dppo {

// Per-kernel timing (dppo_set_timing): while a timed bracket is open (capi.cpp), launches go
// through hipExtLaunchKernel with the bracket's events, which the runtime stamps with the
// kernel's own start and end -- no marker packets in the stream, so short kernels are timed as
// rocprofv3 times them.  The first launch of a bracket takes the start event; every launch takes
// the stop event (the last one's end wins).
struct LaunchTiming {
  hipEvent_t start = nullptr;
  hipEvent_t stop = nullptr;
};
extern thread_local LaunchTiming g_launch_timing;

#define DPPO_LAUNCH(K, G, B, SH, S, ...)                                          \
  do {                                                                            \
    ::dppo::LaunchTiming& lt_ = ::dppo::g_launch_timing;                          \
    if (lt_.stop) {                                                               \
      hipExtLaunchKernelGGL(K, G, B, SH, S, lt_.start, lt_.stop, 0, __VA_ARGS__); \
      lt_.start = nullptr;                                                        \
    } else {                                                                      \
      hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                            \
    }                                                                             \
  } while (0)

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// tanh of two activations: t = e^{-2|x|} = 2^{|x| (-2 log2 e)} (the same bits as __expf(-2|x|):
// scaling by 2 commutes with the rounding), tanh = sign(x) (1 - t) / (1 + t) with one hardware
// reciprocal; the non-transcendental steps run as packed-f32 ops on the pair (v_pk_mul/add_f32).
// Absolute error <= ~1.5e-7 (1 - t cancels near 0: relative, not absolute, accuracy is lost).
__device__ __forceinline__ f32x2 tanh2(f32x2 x) {
  constexpr float kM2Log2e = -2.0f * 1.44269504088896340736f;
  const f32x2 ax = {__builtin_fabsf(x[0]), __builtin_fabsf(x[1])};
  const f32x2 y = ax * kM2Log2e;
  const f32x2 t = {__builtin_amdgcn_exp2f(y[0]), __builtin_amdgcn_exp2f(y[1])};
  const f32x2 d = t + 1.0f;
  const f32x2 r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  const f32x2 q = (1.0f - t) * r;
  return {__builtin_copysignf(q[0], x[0]), __builtin_copysignf(q[1], x[1])};
}

// Launchers implemented in the .hip files (all stream-ordered, no host sync).
int launch_gae_stream_probe(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
                            const float* nv, float* adv, float* ret, int64_t n, hipStream_t s);
int launch_gae(const float* r, const uint8_t* te, const uint8_t* tr, const float* v,
               const float* nv, float* adv, float* ret, double* partials, int T, int N,
               float gamma, float gae_lambda, hipStream_t s, int* n_partials,
               int mode = DPPO_GAE_EXACT);
int launch_stats_reduce(const double* partials, int n_partials, double* dsum, hipStream_t s);
int launch_stats_finalize(const double* dsum, double n_total, float* mean_std, hipStream_t s);
int launch_adv_normalize(float* adv, const float* mean_std, int64_t n, hipStream_t s);

struct PackArgs {
  const float* obs;       // [B][D]
  const void* actions;    // int32 [B] or float [B][A]
  const float* logp;      // [B]
  const float* adv;       // [B] raw advantages
  const float* ret;       // [B]
  const double* dsum;     // {sum, sumsq} of raw advantages (global), or null if no norm
  // single rank: the GAE kernel's per-workgroup {sum, sumsq} partials, reduced by every pack
  // block itself (the same fixed order as stats_reduce_kernel) instead of by a launch of its
  // own; null -> dsum (multi-rank: dsum holds the all-reduced sums)
  const double* partials;
  int n_partials;
  double n_total;         // global sample count for the statistics
  int advantage_norm;
  float* adv_out;         // optional [B]: the (normalised) advantages handed to the update
  float* rec;             // [B][R]
  int64_t B;
  int D, D8, A, R, continuous;
};
int launch_pack(const PackArgs& a, hipStream_t s);

// reduce_adam_kernel's arrival words: [0] top counter, [32 (1 + x)] the counter of XCD group x
// (blockIdx % 8), [32 * 9] the release word; each on its own 128-B line
constexpr int kArrivalWords = 32 * 10;

// ---- optimizer element ops shared by optim.hip and the fused minibatch kernel's tail
// adam_elem on registers (same operations, same order)
__device__ __forceinline__ void adam_regs(float& p, float gr, float& mk, float& vk, float coef,
                                          float w1, float w2, float beta2, float bc2_sqrt,
                                          float eps, float neg_step_size) {
#pragma clang fp contract(off)
  const float g = gr * coef;
  mk = mk + w1 * (g - mk);
  vk = vk * beta2;
  vk = vk + (w2 * g) * g;
  const float denom = sqrtf(vk) / bc2_sqrt + eps;
  p = p + neg_step_size * (mk / denom);
}

__device__ __forceinline__ float clip_coef(double sumsq, float max_norm, float* norm_out) {
  const float norm = (float)sqrt(sumsq);
  // clip_coef = max_norm / (total_norm + 1e-6), clamped to 1, always applied (clip_grad.py:165-169)
  float coef = max_norm / (norm + 1e-6f);
  *norm_out = norm;
  return coef < 1.0f ? coef : 1.0f;
}

// s_pi, s_v, s_h: the loss slots {sum l_pi, sum l_v, sum H} that follow the gradient
__device__ __forceinline__ void write_trace(float* trace, float s_pi, float s_v, float s_h,
                                            float norm, float inv_m, float vf, float ent) {
  const float lpi = s_pi * inv_m;
  const float lv = s_v * inv_m;
  const float h = s_h * inv_m;
  trace[0] = lpi + vf * lv - ent * h;  // ppo.py:276-280
  trace[1] = lpi;
  trace[2] = lv;
  trace[3] = h;
  trace[4] = norm;
}

// Sticky device-side error word of a handle: host-coherent pinned memory (hipHostMallocCoherent,
// mapped), written by kernels with system-scope vector stores and read by the host at the start
// of the next C-ABI call without any synchronisation (capi.cpp device_status).
constexpr unsigned kErrFaninTimeout = 1u;  // a grid-wide fan-in gave up waiting: grid not resident
constexpr unsigned kErrPeerTimeout = 2u;   // a peer exchange gave up waiting for another rank
constexpr unsigned kErrTagTimeout = 3u;    // reduce_adam's tagged-word fan-in gave up waiting
// The word: bits 0-7 the code, 8-15 a rank, 16-31 an index (block, word or slice) -- the wait
// that gave up, so a host report names WHICH wait stalled, not only its kind.
// A wait that runs out of time records its word only when the word is still clear (one
// compare-and-swap), and a wait that finds the word already set leaves without writing: the
// first cause is what the host reads.
__device__ __forceinline__ unsigned err_word(unsigned code, unsigned rank, unsigned idx) {
  return code | (rank & 0xffu) << 8 | (idx & 0xffffu) << 16;
}
__device__ __forceinline__ bool raise_err(unsigned* err, unsigned code) {
  unsigned expect = 0u;  // one compare-and-swap: of two waves timing out together, the first wins
  return __hip_atomic_compare_exchange_strong(err, &expect, code, __ATOMIC_RELAXED,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The first cause's evidence (words 2-3 of the 64-B error block): the last value the stalled wait
// read, written only by the wait that won raise_err.
__device__ __forceinline__ void raise_err_seen(unsigned* err, unsigned code,
                                               unsigned long long seen) {
  if (raise_err(err, code)) {
    __hip_atomic_store(err + 2, (unsigned)seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(err + 3, (unsigned)(seen >> 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__device__ __forceinline__ bool err_set(const unsigned* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}
// Default bound of one fan-in wait, in s_memrealtime ticks (100 MHz): 5 s.  A resident grid
// arrives within microseconds; only a grid that is NOT co-resident (another process holding CUs
// with a long kernel, a partitioned device) can wait this long.
constexpr unsigned long long kFaninTimeoutTicks = 500000000ull;

// Grid-wide fan-in by thread 0 of each workgroup: arrive on the counter of this block's XCD group
// (blockIdx % 8), the last arriver of a group adds to the top counter, the last of those writes
// the release word that every block polls.  Counters are monotonic: launch `epoch` (1, 2, ...)
// waits for epoch x arrivals.  The caller drains its publishing stores (vmcnt(0)) before, and
// reads handed-off data with sc1 loads after.
//
// Returns false -- and sets *err to kErrFaninTimeout -- when the release has not come after
// `timeout_ticks` of wall clock, or as soon as *err is already set (an earlier fan-in of this
// handle failed: queued launches then drain in ~256 polls each instead of waiting out their own
// timeouts).  The caller must then NOT use the handed-off data.  Every block reaches an exit:
// the grid always drains, resident or not.
__device__ __forceinline__ bool grid_fanin(unsigned* ctr, unsigned epoch,
                                           unsigned long long timeout_ticks, unsigned* err) {
  const unsigned x = blockIdx.x & 7;
  const unsigned nx = (gridDim.x - x + 7) / 8;
  const unsigned ng = gridDim.x < 8 ? gridDim.x : 8;
  unsigned* rel = ctr + 32 * 9;
  const unsigned o1 =
      __hip_atomic_fetch_add(ctr + 32 * (1 + x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (o1 == epoch * nx - 1) {
    const unsigned o2 = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o2 == epoch * ng - 1) __hip_atomic_store(rel, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned k = 0;
       (int)(__hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - epoch) < 0; ++k) {
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255u) == 255u) {
      const bool late = __builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks;
      if (late || err_set(err)) {
        if (late) raise_err(err, err_word(kErrFaninTimeout, 0u, blockIdx.x));
        return false;
      }
    }
  }
  return true;
}

// Default actor-critic MLP (hidden 64) kernels: mlp.hip.
struct MlpShape {
  int D, D8, A, continuous, R;  // R = record stride (floats)
};
size_t mlp_lds_bytes_eval(const MlpShape& sh);
// Next-value reuse of the old-policy evaluation over a [T][row] rollout: where next_obs[i] is
// bitwise obs[i + row], V(next_obs[i]) = values[i + row]; only the other samples get a critic
// pass of their own, run by the eval kernel's waves from a wave-private LDS ring (no second
// launch).  Results are bit-identical to the full evaluation.
struct EvalReuse {
  int64_t row;  // > 0: the buffers are a [T][row] rollout, next_obs[i] may be obs[i + row]
};
int launch_eval(const MlpShape& sh, const ParamOffsets& po, const float* params, const float* obs,
                const void* actions, const float* next_obs, float* logp, float* values,
                float* next_values, int64_t n, hipStream_t s, EvalReuse* reuse = nullptr);
// optional env-action output of the continuous act kernel: tanh(u), rescaled to [low, high]
// when both bound arrays are given (host arrays of A floats)
struct ActSquash {
  float* env_actions;
  const float* low;
  const float* high;
};
int launch_act(const MlpShape& sh, const ParamOffsets& po, const float* params, const float* obs,
               void* actions, int64_t n, uint64_t seed, uint64_t counter, hipStream_t s,
               float* heads = nullptr, const ActSquash* squash = nullptr);
struct GradArgs {
  const float* params;
  const float* rec;
  const int32_t* idx;  // minibatch sample indices (local)
  const int32_t* seg;  // or null; else device {start, end}: the minibatch is idx[start, end)
  int32_t m;           // samples in this minibatch on this rank (ignored when seg is set)
  float inv_m;         // 1 / global minibatch size
  float clip_eps, vf_coef, ent_coef;
  float* slabs;        // [G][slab_stride]
  int64_t slab_stride; // floats per slab (param total + 8 loss slots, rounded)
  int64_t p_total;
};
// Single-device tail of the fused minibatch kernel: slab reduction, clip_grad_norm_ and Adam in
// the same launch (two grid-wide fan-ins instead of a second launch), see mbstep.hip.
struct FusedAdam {
  float* grad;          // [p_total + 8] reduced gradient + loss slots (published sc1)
  double* sq_part;      // [nblk] per-64-parameter-block sums of squares
  unsigned* arrivals;   // 2 x kArrivalWords (two fan-ins)
  unsigned epoch;       // launch number (monotonic counters, never reset)
  unsigned* err;        // sticky device error word (host-coherent), see grid_fanin
  unsigned long long timeout_ticks;
  float* params;        // updated in place
  float* m;
  float* v;
  float max_norm, neg_step_size, bc2_sqrt, beta1, beta2, eps;
  float* trace;         // [5] {loss, l_pi, l_v, H, norm} of this minibatch
  int64_t ls_off;       // continuous: log-std parameters get -entropy_beta added (optim.hip)
  int ls_n;
  int add_entropy_const;
};
// Fused minibatch kernels.  launch_mb runs the sample-split kernel (mbwave.hip: one wave per
// SIMD, heads on VALU, up to 4 actions) where it applies and the feature-split two-team kernel
// (mbstep.hip) otherwise -- more actions, the fused Adam tail, or DPPO_MB_LEGACY=1.  mb_grid
// gives the workgroup count (= gradient slabs) of the kernel launch_mb will run.
size_t mb_lds_bytes(const MlpShape& sh);
int mb_grid(const MlpShape& sh, int32_t m, bool fused = false);
int launch_mb(const MlpShape& sh, const ParamOffsets& po, const GradArgs& a, int G,
              hipStream_t s, const FusedAdam* fused = nullptr);
bool mbw_supported(const MlpShape& sh);
int mbw_grid(int32_t m);
size_t mbw_lds_bytes(const MlpShape& sh);
int launch_mbw(const MlpShape& sh, const ParamOffsets& po, const GradArgs& a, int G,
               hipStream_t s);

// Optimiser kernels: optim.hip.
int slab_reduce_blocks(int64_t p_total);
int launch_slab_reduce(const float* slabs, int G, int64_t slab_stride, int64_t p_total,
                       float* grad, double* sq_part, int64_t ls_off, int ls_n, float ent_coef,
                       int add_entropy_const, hipStream_t s);
int launch_clip_adam_traced(float* params, float* grad, float* m, float* v, int64_t n,
                            const double* sq_part, int n_sq, float max_norm, float neg_step_size,
                            float bc2_sqrt, float beta1, float beta2, float eps, float* out_norm,
                            float* trace, float inv_m, float vf, float ent, hipStream_t s);
// slab reduce + clip + Adam fused (single device): `tags` = reduce_adam_tag_words(p_total)
// 64-bit words zeroed once; launch number `epoch` (1, 2, ...) publishes and waits for words
// tagged `epoch`.  On a wait timeout the blocks leave their parameters untouched and set *err.
struct PeerArgs;
// `peer` (may be null): sum each block's gradient slice over the ranks of a peer exchange before
// the norm (peer.hip; src / dst / n unused, seq = this exchange's number)
int launch_reduce_adam(const float* slabs, int G, int64_t slab_stride, int64_t p_total, float* grad,
                       unsigned long long* tags, int64_t ls_off, int ls_n, float ent_coef,
                       int add_entropy_const, unsigned epoch, float* params,
                       float* m, float* v, float max_norm, float neg_step_size, float bc2_sqrt,
                       float beta1, float beta2, float eps, float* trace, float inv_m, float vf,
                       float ent, unsigned* err, unsigned long long timeout_ticks, hipStream_t s,
                       const PeerArgs* peer = nullptr);
// Workgroups of reduce_adam_kernel that fit on the device at once (occupancy x CUs; 0 when the
// layout has more tagged words than the kernel's polling wave holds).
int reduce_adam_capacity(int device, int64_t p_total);
int reduce_adam_blocks(int64_t p_total);
int reduce_adam_tag_words(int64_t p_total);
// Fan-in self test (dppo_fanin_selftest): `blocks` workgroups of 1024 threads holding
// `lds_bytes` of LDS each meet in one grid_fanin on `ctr` (zeroed by the caller, epoch 1).
int launch_fanin_probe(int blocks, int lds_bytes, unsigned* ctr, unsigned* err,
                       unsigned long long timeout_ticks, hipStream_t s);
int launch_clip_adam(float* params, float* grad, float* m, float* v, int64_t n, float max_norm,
                     float neg_step_size, float bc2_sqrt, float beta1, float beta2, float eps,
                     float* out_norm, hipStream_t s);
// out[i] = src[0][i] + src[1][i] + ... + src[n-1][i] in rank order (f32 or f64 when `f64`); the
// device-local stand-in for the RCCL sum of a single-device loopback group (capi.cpp)
constexpr int kMaxLoopRanks = 8;

// Peer exchange (peer.hip): one-shot all-reduce over the ranks' mapped exchange buffers.
constexpr int kMaxPeers = 8;
constexpr int kPeerChunk = 1024;      // elements per workgroup (one flag each)
constexpr int kPeerMaxSlices = 64;    // up to 65,536 elements per exchange
struct PeerArgs {
  const void* src;        // this rank's vector (n elements)
  void* dst;              // the rank-ordered sum (may alias src)
  char* bufs[kMaxPeers];  // every rank's exchange buffer as mapped in this process
  int64_t n;
  int64_t data_bytes;     // bytes of one parity's data region
  int world, rank;
  unsigned seq;           // exchange number, the same sequence on every rank (1, 2, ...)
  unsigned* err;          // the handle's sticky device error word
  unsigned long long timeout_ticks;
  int acq;                // diagnosis (DPPO_TEST_HOOKS + DPPO_PEER_ACQ=1): a system-scope acquire
                          // fence before every poll of a peer word
};
int64_t peer_buffer_bytes(int64_t cap);  // cap = elements (of up to 8 B) per parity
int launch_peer_sum(const PeerArgs& a, bool f64, hipStream_t s);

// Exchange buffer of rank r (each region data_bytes = cap x 8 B):
//   [values, parity 0][values, parity 1][tagged words, parity 0][tagged words, parity 1]
//   [kPeerMaxSlices slice flags, 64 B apart]
// Values + slice flags: peer_sum_kernel (any element type).  Tagged words {seq, float}: the
// gradient exchange inside reduce_adam_kernel, where the data is its own arrival flag.  Data moves
// with system-scope (sc0 sc1) stores and loads: coherent across GPUs on their own, no L2
// write-back or invalidate (peer.hip).
__device__ __forceinline__ unsigned* peer_flag(const PeerArgs& a, int r, int slot) {
  return (unsigned*)(a.bufs[r] + 4 * a.data_bytes + 64 * (int64_t)slot);
}
__device__ __forceinline__ unsigned long long* peer_tagged(const PeerArgs& a, int r) {
  return (unsigned long long*)(a.bufs[r] + (2 + (int64_t)(a.seq & 1u)) * a.data_bytes);
}
template <typename T>
__device__ __forceinline__ void peer_put(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T peer_get(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Wait until *f reaches a.seq (wrap-safe); false -- with kErrPeerTimeout raised -- after
// a.timeout_ticks of wall clock or once the handle's error word is already set.
__device__ __forceinline__ bool peer_wait(const unsigned* f, const PeerArgs& a, int r, int slot) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned k = 0;; ++k) {
    if (a.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - a.seq) >= 0)
      break;
    __builtin_amdgcn_s_sleep(1);
    if ((k & 255u) == 255u) {
      const bool late = __builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks;
      if (late || err_set(a.err)) {
        if (late)
          raise_err_seen(a.err, err_word(kErrPeerTimeout, (unsigned)r, (unsigned)slot),
                         __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        return false;
      }
    }
  }
  return true;
}
struct RankPtrs {
  const void* p[kMaxLoopRanks];
};
int launch_rank_sum(const RankPtrs& src, int n, void* out, int64_t count, bool f64,
                    hipStream_t s);

// RecurrentPPO fused minibatch gradient (gru.hip): parameter offsets in the flat layout
// (RecurrentActorCriticNetwork.named_parameters() order) and the per-sample scratch arrays.
struct GruOffsets {
  int64_t Wb, bb, Wih, Whh, bih, bhh, Wa1, ba1, Wa2, ba2, Wc1, bc1, Wc2, bc2;
};
struct GruScratch {
  float *obs, *x1, *gi, *hi, *ho, *r, *z, *n, *ghn, *ya, *yc, *dl, *dv, *dya, *dyc, *dho, *dgi,
      *dgh, *dx1;
};
size_t gru_lds_bytes(int D);
int gru_grid(int N);
int launch_gru_grad(const GruOffsets& po, const float* params, const dppo_gru_batch& b,
                    const int32_t* idx, int32_t m, float* wmask, int64_t B, int T, int N, int D,
                    int A, float inv_m, float clip_eps, float vf, float ent, const GruScratch& sc,
                    float* slabs, int64_t slab_stride, int64_t p_total, hipStream_t s);

// Fisher-Yates resolution (shuffle.hip): perms[c][n] from swap targets[c][n]; scratch of
// scratch_ints >= 3 * count * n int32 (perm_scratch_ints: the size at which the partitioned
// buckets run fused).
int64_t perm_scratch_ints(int64_t n, int32_t count);
int launch_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                        int32_t* scratch, int64_t scratch_ints, hipStream_t s);

// Global-minibatch data parallelism (shuffle.hip): from E global permutations gperm[E][T*Ng]
// keep, in order, the samples of env shard [env0, env0 + Nl) as local indices t*Nl + (n - env0)
// into local[E][T*Nl]; seg[E][M+1] = where each global minibatch (mbg samples) starts in the
// epoch's list.  cnt: scratch of E * shard_select_chunks(T*Ng) ints.
// Global minibatches straight from the swap targets: bucket build + a value walk of this rank's
// samples only + the ordered selection (no whole-permutation resolution).  DPPO_PERM_WALK=0:
// resolve + select instead (A/B).
bool perm_walk();
int launch_shard_select_targets(const int32_t* targets, int32_t* marks, int32_t* scratch,
                                int64_t scratch_ints, int32_t* local, int32_t* seg, int32_t* cnt,
                                int64_t bg, int32_t ng, int32_t env0, int32_t nl, int32_t E,
                                int32_t M, hipStream_t s);
int shard_select_chunks(int64_t bg);
int launch_shard_select(const int32_t* gperm, int32_t* local, int32_t* seg, int32_t* cnt,
                        int64_t bg, int32_t ng, int32_t env0, int32_t nl, int32_t E, int32_t M,
                        hipStream_t s);

// ---- Wave-wide f64 reductions (GAE statistics partials, the optimizer's global norm)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double lane_f64(double x, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Wave sum in a fixed order, the result valid in every lane: DPP within each 16-lane row (xor 1,
// xor 2, half-row mirror, row mirror: VALU data moves, no LDS round trip), then the 4 row sums
// read from lanes 0/16/32/48.  Replaces a 6-round ds_bpermute butterfly that sat at the end of
// the launch, after the last stores.
__device__ __forceinline__ double wave_sum_f64(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f64<0x141>(x);  // row_half_mirror
  x += dpp_f64<0x140>(x);  // row_mirror
  return (lane_f64(x, 0) + lane_f64(x, 16)) + (lane_f64(x, 32) + lane_f64(x, 48));
}

}  // namespace dppo
