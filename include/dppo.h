/*
 * libdppo -- MI355X (gfx950) native PPO hot path: GAE + clipped-surrogate minibatch update.
 *
 * C ABI (plain pointers and sizes, no torch types).  Every call that touches the GPU is
 * stream-ordered on the caller's hipStream_t (passed as void*; NULL = legacy default stream),
 * performs no host synchronisation unless documented, and never allocates on the hot path:
 * workspace is allocated once by dppo_create().  Handles are reentrant across handles, NOT
 * thread-safe on one handle.  One process per GPU.
 *
 * The reference (Auxeno/diamond-ppo) is pure Python with no FFI; each entry point below names
 * the reference code it replaces (file:line in diamond/).  The Python host mirror that binds
 * this ABI is diamond-ppo_amd/diamond/_native.py (ctypes); see INTEGRATION.md.
 *
 * Layouts (HBM, structure-of-arrays, flat sample index i = t*N + n, reference ppo.py:246-249):
 *   obs, next_obs  float32 [T][N][D]          rewards        float32 [T][N]
 *   term, trunc    uint8   [T][N] (0/1)       actions        int32 [T][N] (discrete) or
 *                                                            float32 [T][N][A] (continuous)
 *   params, adam m/v: one flat float32 buffer each, tensors at dppo_param_layout() offsets.
 *
 * Status codes: 0 = OK, negative = error; dppo_last_error() describes the last failure on the
 * calling thread.  The Python binding maps them to the reference's exception types.
 */
#ifndef DPPO_H_
#define DPPO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* the library is built with -fvisibility=hidden: only these declarations are exported */
#pragma GCC visibility push(default)

#define DPPO_OK 0
#define DPPO_EINVAL (-1)       /* invalid argument (Python: ValueError / AssertionError) */
#define DPPO_EHIP (-2)         /* HIP runtime error (Python: RuntimeError) */
#define DPPO_EUNSUPPORTED (-3) /* shape outside the fused kernels' support (Python: NotImplementedError) */
#define DPPO_ENOMEM (-4)       /* workspace allocation failed (Python: MemoryError) */
#define DPPO_ECOMM (-5)        /* RCCL failure (Python: RuntimeError) */

/* GAE modes (dppo_set_gae_mode): the reference's serial recurrence, bit-exact (default); or the
 * chunked affine scan, within 1e-6 of the advantages' scale (SURVEY 7.2 hard part 1). */
#define DPPO_GAE_EXACT 0
#define DPPO_GAE_AFFINE 1

#define DPPO_MAX_TENSORS 16
#define DPPO_TRACE_FIELDS 5 /* per optimizer step: loss, loss_policy, loss_value, entropy, grad_norm */

typedef struct dppo_handle dppo_handle;

/* Shapes.  Mirrors the PPOConfig / ContinuousPPOConfig fields the hot path reads
 * (reference ppo.py:15-37, continuous_ppo.py:15-37) plus the env-axis shard. */
typedef struct dppo_dims {
  int32_t rollout_steps;   /* T */
  int32_t num_envs;        /* N: envs owned by THIS rank */
  int32_t obs_dim;         /* D = prod(observation_space.shape)        (ppo.py:54) */
  int32_t act_dim;         /* discrete: action_space.n; continuous: prod(action_space.shape) */
  int32_t continuous;      /* 0 = PPO/Categorical, 1 = ContinuousPPO/JointNormal */
  int32_t hidden;          /* network_hidden_dim (ppo.py:32,51) */
  int32_t num_epochs;      /* ppo.py:25 */
  int32_t num_minibatches; /* ppo.py:26 */
  int32_t world_size;      /* ranks sharing the env axis (1 = single GPU) */
  int32_t rank;
  /* Minibatch semantics across ranks (world_size > 1 only):
   *  0 = local: each rank permutes its own T*N samples; global minibatch j is the union of the
   *      ranks' local minibatches j (host_perms: [E][T*N] local indices).
   *  1 = global: every rank passes the SAME permutations of the global batch (host_perms:
   *      [E][T*N*world_size], global flat index t*(N*world_size) + n, i.e. what the reference's
   *      np.random.permutation(B) draws for the whole batch, ppo.py:252-255); each rank processes
   *      the members of every global minibatch that fall in its env shard [rank*N, (rank+1)*N).
   *      world_size ranks then reproduce the single-GPU learn of the global batch. */
  int32_t global_minibatches;
} dppo_dims;

/* Hyper-parameters of one learn() call (ppo.py:15-37, Adam defaults torch/optim/adam.py:39). */
typedef struct dppo_hparams {
  float gamma, gae_lambda, ppo_clip, value_loss_weight, entropy_beta, grad_norm_clip;
  float adam_beta1, adam_beta2, adam_eps;
  int32_t advantage_norm;
  double lr;         /* current learning rate (after LinearLR, ppo.py:137-142,287) */
  int64_t adam_step; /* optimizer steps taken before this call (torch Adam state['step']) */
} dppo_hparams;

/* Flat parameter layout, tensors in the reference's named_parameters() order
 * (discrete: base.0.{weight,bias}, base.2.*, actor_head.0.*, actor_head.2.*, critic_head.0.*,
 *  critic_head.2.*; continuous: actor_log_std first, then base, actor_mean_head, critic_head).
 * Each tensor starts on a 64-byte boundary; padding floats are never read as parameters. */
typedef struct dppo_layout {
  int64_t total;  /* floats in the flat buffer, padding included */
  int64_t n_real; /* real parameter count (12,995 for CartPole at hidden 64) */
  int32_t count;  /* number of tensors */
  int32_t pad_;
  int64_t offset[DPPO_MAX_TENSORS];
  int64_t numel[DPPO_MAX_TENSORS];
  int32_t rows[DPPO_MAX_TENSORS]; /* weight [out][in]: rows=out, cols=in; bias: rows=n, cols=1 */
  int32_t cols[DPPO_MAX_TENSORS];
} dppo_layout;

/* Device rollout buffer (caller-owned). */
typedef struct dppo_rollout {
  const float* obs;
  const float* next_obs;
  const void* actions; /* int32 [T][N] or float32 [T][N][A] */
  const float* rewards;
  const uint8_t* term;
  const uint8_t* trunc;
} dppo_rollout;

/* Optional caller-owned device outputs of one learn() (NULL = keep internal).  All [T*N]. */
typedef struct dppo_learn_outputs {
  float* log_probs;   /* old-policy log pi(a|s)                         ppo.py:237 */
  float* values;      /* V(s)                                           ppo.py:236 */
  float* next_values; /* V(s')                                          ppo.py:238 */
  float* advantages;  /* GAE, normalised if advantage_norm              ppo.py:240-243 */
  float* returns;     /* values + raw advantages                        ppo.py:241 */
} dppo_learn_outputs;

const char* dppo_version(void);
const char* dppo_last_error(void);
int dppo_param_layout(const dppo_dims* dims, dppo_layout* out);

/* Workspace sized for dims (rollout buffers, sample records, gradient slabs, trace). */
int dppo_create(int device, const dppo_dims* dims, dppo_handle** out);
void dppo_destroy(dppo_handle* h);

/* GAE over the [T][N] buffers: replaces PPO.calculate_advantage (ppo.py:188-222; identical in
 * continuous_ppo.py:200-234, recurrent_ppo.py:265-299) fused with returns = values + adv
 * (ppo.py:241).  Bit-exact with the reference's fp32 op order.  Also records the per-tile
 * (sum, sum of squares) partials the next call reduces. */
int dppo_gae_f32(dppo_handle* h, const float* rewards, const uint8_t* term, const uint8_t* trunc,
                 const float* values, const float* next_values, float* adv, float* returns,
                 float gamma, float gae_lambda, void* stream);

/* Select the GAE kernel of this handle's dppo_gae_f32 / dppo_learn_f32 calls: DPPO_GAE_EXACT
 * (default; bit-exact with ppo.py:197-220) or DPPO_GAE_AFFINE (chunk maps composed in parallel;
 * re-associated fp32, <= 1e-6 of the advantages' scale from the reference). */
int dppo_set_gae_mode(dppo_handle* h, int32_t mode);

/* Measurement only (no reference counterpart): the streaming ceiling of dppo_gae_f32 -- the same
 * 22 bytes per element over the same buffers (reads rewards, values, next_values, term, trunc;
 * writes adv and returns with meaningless values), no recurrence, one persistent grid.  Timed
 * like the GAE kernel (dppo_set_timing, class "gae_probe").  T*N % 4 == 0, 16-B aligned buffers. */
int dppo_gae_stream_probe(dppo_handle* h, const float* rewards, const uint8_t* term,
                          const uint8_t* trunc, const float* values, const float* next_values,
                          float* adv, float* returns, void* stream);

/* Mean and unbiased std of the advantages of the last dppo_gae_f32 (ppo.py:243, reduced over
 * all ranks when a communicator is attached); writes device float mean_std[2]. */
int dppo_adv_stats(dppo_handle* h, float* mean_std, void* stream);

/* The pieces of dppo_adv_stats for a caller that does its own exchange (RecurrentPPO under
 * torch.distributed): dppo_adv_sums writes this rank's {sum adv, sum adv^2} of the last
 * dppo_gae_f32 as device double[2]; after the caller's all-reduce, dppo_adv_stats_from_sums turns
 * the global sums of n_total advantages into the mean and unbiased std (ppo.py:243). */
int dppo_adv_sums(dppo_handle* h, double* sums, void* stream);
int dppo_adv_stats_from_sums(const double* sums, double n_total, float* mean_std, void* stream);

/* adv = (adv - mean) / (std + 1e-6) in place (ppo.py:243). */
int dppo_adv_normalize_f32(float* adv, const float* mean_std, int64_t n, void* stream);

/* Old-policy evaluation with the default actor-critic MLP (ppo.py:235-238 with
 * ActorCriticNetwork ppo.py:53-96; continuous_ppo.py:247-250 with :63-111): log-prob of the
 * taken actions, V(obs), V(next_obs).  n samples; obs/next_obs [n][D]; actions int32 [n] or
 * float32 [n][A]. */
int dppo_old_policy_f32(dppo_handle* h, const float* params, const float* obs, const void* actions,
                        const float* next_obs, float* log_probs, float* values, float* next_values,
                        int64_t n, void* stream);

/* Rollout action sampling with the default actor MLP (replaces get_actions, ppo.py:73-82:
 * Categorical(logits).sample(); continuous_ppo.py:83-93: Normal(mean, exp(log_std)).sample()).
 * obs [n][D] on the device; actions out int32 [n] or float32 [n][A].  Randomness: Philox4x32-10
 * keyed by `seed`, counter (sample index, `counter`) -- deterministic for a given
 * (seed, counter), the same distribution as the reference's torch draws but not the same draws;
 * advance `counter` once per call. */
int dppo_act_f32(dppo_handle* h, const float* params, const float* obs, int64_t n, uint64_t seed,
                 uint64_t counter, void* actions, void* stream);

/* dppo_act_f32 for a continuous action space, plus the action the environment receives under
 * the tanh-squash option (an extension -- the reference sends the raw Gaussian
 * sample, continuous_ppo.py:83-93): actions [n][A] = the Gaussian samples u (the same draws as
 * dppo_act_f32 for this seed / counter; the experience keeps them), env_actions [n][A] =
 * low + (tanh(u) + 1) * (high - low) / 2 with low/high host arrays of A finite floats (high > low),
 * or tanh(u) when both are NULL. */
int dppo_act_squash_f32(dppo_handle* h, const float* params, const float* obs, int64_t n,
                        uint64_t seed, uint64_t counter, const float* low, const float* high,
                        float* actions, float* env_actions, void* stream);

/* The actor half of dppo_act_f32 without the draw: the logits (discrete, ppo.py:79) or Gaussian
 * means (continuous, continuous_ppo.py:88-90) of the default actor for obs [n][D], written to
 * heads [n][A] -- exactly the values dppo_act_f32 samples from. */
int dppo_actor_forward_f32(dppo_handle* h, const float* params, const float* obs, int64_t n,
                           float* heads, void* stream);

/* One full PPO.learn (ppo.py:224-287 / continuous_ppo.py:236-299) with the default network:
 * old-policy eval, GAE, returns, advantage normalisation, then num_epochs x num_minibatches
 * {gather, forward, clipped-surrogate + value + entropy loss, analytic backward, [RCCL
 * all-reduce], clip_grad_norm_, Adam}.  perms: host int32 [E][T*N] (np.random.permutation
 * output per epoch, ppo.py:254), copied asynchronously through pinned staging.  params/m/v are
 * updated in place.  Asynchronous: returns once everything is enqueued on `stream`.  Returns
 * DPPO_EINVAL if T*N is not divisible by num_minibatches (the reference's reshape raises). */
int dppo_learn_f32(dppo_handle* h, const dppo_rollout* rollout, float* params, float* adam_m,
                   float* adam_v, const dppo_hparams* hp, const int32_t* host_perms,
                   const dppo_learn_outputs* outputs, void* stream);

/* dppo_learn_f32 with the permutations given as their Fisher-Yates swap targets (host int32
 * [E][T*N], dppo_perm_targets_numpy output): the shuffle itself is resolved on the device
 * (dppo_perm_resolve), so the host only runs the MT19937 draws.  Same results bit for bit. */
int dppo_learn_targets_f32(dppo_handle* h, const dppo_rollout* rollout, float* params,
                           float* adam_m, float* adam_v, const dppo_hparams* hp,
                           const int32_t* host_targets, const dppo_learn_outputs* outputs,
                           void* stream);

/* Gradient of the minibatch loss at `params` for samples idx[0..m) of the records built by
 * the last dppo_learn_f32/dppo_prepare_f32 (ppo.py:261-283), written to grad[P] (flat layout,
 * unclipped), plus, if loss4 is non-NULL, the loss terms to HOST loss4[4] = {loss, loss_policy,
 * loss_value, entropy} (synchronises the stream).  idx: device int32.  m_total: divisor of the
 * means (global minibatch size). */
int dppo_minibatch_grad_f32(dppo_handle* h, const float* params, const int32_t* idx, int32_t m,
                            int32_t m_total, const dppo_hparams* hp, float* grad, float* loss4,
                            void* stream);

/* Stage a rollout for dppo_minibatch_grad_f32 without updating: old-policy eval, GAE, returns,
 * normalisation, sample records (the first half of dppo_learn_f32). */
int dppo_prepare_f32(dppo_handle* h, const dppo_rollout* rollout, const float* params,
                     const dppo_hparams* hp, const dppo_learn_outputs* outputs, void* stream);

/* clip_grad_norm_ (ppo.py:284, torch nn/utils/clip_grad.py) + Adam step (ppo.py:285, torch
 * optim/adam.py _single_tensor_adam) over a flat buffer of n floats; step = step count AFTER
 * this update.  Optional out_norm (device float) receives the pre-clip total norm. */
int dppo_clip_adam_f32(float* params, float* grad, float* adam_m, float* adam_v, int64_t n,
                       float max_norm, double lr, float beta1, float beta2, float eps, int64_t step,
                       float* out_norm, void* stream);

/* One of the handle's DPPO_PERM_SLOTS (3) pinned host staging buffers (slot 0..2) for the
 * [E][T*N] permutations or swap targets; waits for the previous learn's upload from that slot to
 * finish.  Generating straight into a slot (dppo_perm_numpy / dppo_perm_targets_numpy) and
 * passing it to dppo_learn_f32 / dppo_learn_targets_f32 makes the upload a pure asynchronous DMA;
 * three slots let the draws of the next two learns run on the host while the current learn's
 * upload is in flight. */
#define DPPO_PERM_SLOTS 3
int dppo_perm_buffer(dppo_handle* h, int32_t slot, int32_t** out);

/* External staging slots (round 5): caller-owned host memory of `bytes` (e.g. a slot of a
 * node-shared draw in POSIX shared memory) page-locked by the handle (hipHostRegister) as slot
 * k (0..DPPO_PERM_EXT_SLOTS-1), so that dppo_learn_f32 / dppo_learn_targets_f32 given that
 * pointer upload from it directly; ptr = NULL unregisters (after the slot's last upload).
 * dppo_perm_external_done: *done = 1 once the last upload from slot k has completed (a
 * non-blocking event query).  Replaces nothing in the reference: the shared-draw plumbing of
 * ppo.py:252-255 across a node's ranks. */
#define DPPO_PERM_EXT_SLOTS 8
int dppo_perm_external(dppo_handle* h, int32_t k, int32_t* ptr, int64_t bytes);
int dppo_perm_external_done(dppo_handle* h, int32_t k, int32_t* done);

/* Per-kernel timing with HIP events (off by default): while enabled, every kernel the handle
 * launches carries a start/stop event pair stamped with the kernel's own execution interval
 * (hipExtLaunchKernel), RCCL calls a pair of stream markers.  Classes, in order: old-policy eval,
 * GAE, advantage-stat reduce, record pack, fused minibatch gradient, slab reduce, clip+Adam, RCCL
 * all-reduce, Fisher-Yates resolution, fused slab reduce + clip + Adam (single device).
 * dppo_set_timing() synchronises the device and clears the records; dppo_get_timing()
 * synchronises and returns per-class summed milliseconds and launch counts. */
#define DPPO_TIMING_CLASSES 10
int dppo_set_timing(dppo_handle* h, int32_t enable);
int dppo_get_timing(dppo_handle* h, double* ms_sum, int64_t* counts);

/* Per-step trace of the last dppo_learn_f32: E*M rows of DPPO_TRACE_FIELDS floats, copied to
 * host memory.  Synchronises the handle's stream. */
int dppo_get_trace(dppo_handle* h, float* host_out, int32_t rows);

/* NumPy legacy RandomState.permutation, bit-exact (ppo.py:254): `count` permutations of
 * arange(n) into out[count][n], advancing the MT19937 key[624]/pos in place exactly as
 * np.random.permutation would.  Host only. */
int dppo_perm_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out);

/* dppo_perm_numpy in two halves: returns once the draws are done (key / pos already advanced, so
 * the next learn's draws may start) while the Fisher-Yates swaps finish on the host worker pool;
 * dppo_perm_wait(ticket) waits for them (out is complete afterwards) and frees the ticket.  Every
 * ticket must be waited for exactly once.  Host only. */
int dppo_perm_numpy_async(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out,
                          void** ticket);
int dppo_perm_wait(void* ticket);

/* Counters of the host permutation draws since load: {calls, calls whose Fisher-Yates swaps ran
 * on the pinned swap pool, calls whose MT19937 blocks came from the producer thread's ring}.
 * DPPO_PERM_PIN=3 pins the pool to every allowed CPU (no cache-topology lookup). */
int dppo_perm_stats(int64_t* out3);

/* Host placement of the permutation draws (host only; no reference counterpart -- the reference
 * draws on its own Python thread, diamond/ppo.py:254).  The swap pool and the drawing thread run
 * in one L3 domain, chosen at first use as the least busy one by a /proc/stat sample
 * (DPPO_PERM_BY_LOAD=0: CPU order).  dppo_perm_repin chooses again (a ~25 ms sample; call it off
 * the launching thread) and moves the pool at its next job: out4 (nullable) = {moved, first CPU of
 * the domain, its busy % when chosen, re-pins so far}.  dppo_perm_domain reports the last three
 * without sampling. */
int dppo_perm_repin(int64_t* out4);
int dppo_perm_domain(int64_t* out3);

/* The MT19937 half of dppo_perm_numpy: the Fisher-Yates swap targets out[c][i] = j_i
 * (i = n-1 .. 1; out[c][0] = 0) of `count` successive permutations, advancing key/pos exactly
 * as dppo_perm_numpy does.  Host only.  Draws of >= 2^22 targets run the parallel form below on
 * DPPO_PERM_PAR_THREADS threads (default 12; < 2 = serial). */
int dppo_perm_targets_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out);

/* The same draw split over `threads` threads (csrc/permpar.cpp: MT19937 jump-ahead, a
 * speculative accept scan per chunk of the word stream, an exact serial stitch, a parallel
 * assembly); identical outputs and key/pos advance.  Falls back to the serial draw (never to a
 * different result) when a stitch check fails.  opts (nullable, 3 x int64): chunks (0 = threads),
 * near-miss band W (0 = 4 sigma of the model), W multiplier x100 (0 = 400).  stats (nullable,
 * 24 x int64): [0] path (0 serial, 1 parallel, 2 parallel attempt fell back), [1] chunks,
 * [2] near-miss records, [3] kept zone words, [4] replayed words, [5] max |offset|, [6] W,
 * [7] Wb, [8] scan us, [9] stitch us, [10] assembly us, [11] slowest chunk us, [12] words
 * generated, [13] failure code, [14] total us, [15] slowest jump-ahead us, [16] words scanned
 * one at a time, [17] disagreeing words applied, [18] µs the stitch worked (its waits for chunk
 * scans excluded).  Host only.
 * Replaces the serial draw behind reference diamond/ppo.py:252-255 (np.random.permutation). */
int dppo_perm_targets_numpy_par(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                                int32_t* out, int32_t threads, const int64_t* opts,
                                int64_t* stats);

/* Parallel-draw counters since load: {attempts by dppo_perm_targets_numpy, parallel draws
 * completed, fallbacks to the serial draw}. */
int dppo_perm_par_stats(int64_t* out3);

/* The swap half on the device: perms[c] = arange(n) shuffled by targets[c] (device int32
 * [count][n]), identical to the sequential Fisher-Yates loop.  scratch: device int32
 * [3 * count * n].  Stream-ordered.  (A handle's own resolution, dppo_learn_targets_f32, uses a
 * larger internal scratch that lets its bucket sort store one packed word per step.) */
int dppo_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                      int32_t* scratch, void* stream);
/* dppo_perm_resolve with the scratch size given (int32 elements, >= 3 * count * n): from
 * dppo_perm_resolve_scratch(n, count) up, the bucket sort stores one packed word per step and
 * fuses its bucket pass in LDS (the handle's own form; ~1.8x faster at 4 x 8.4 M).  Same results
 * bit for bit.  dppo_perm_resolve_scratch returns -1 on invalid sizes. */
int64_t dppo_perm_resolve_scratch(int64_t n, int32_t count);
int dppo_perm_resolve_ex(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                         int32_t* scratch, int64_t scratch_ints, void* stream);

/* Global minibatches on the device (dims.global_minibatches, world_size > 1): from the swap
 * targets of the GLOBAL batch (device int32 [E][T*N*world_size], dppo_perm_targets_numpy of
 * B*world_size), this rank's members of every global minibatch in permutation order as local
 * sample indices (device int32 local[E][T*N]) and each epoch's minibatch boundaries (device
 * int32 seg[E][M+1]).  Only this rank's samples are walked to their positions (the whole
 * permutation is never resolved; DPPO_PERM_WALK=0: resolve, then select).  What
 * dppo_learn_targets_f32 does before its minibatch steps (reference ppo.py:252-255 + the
 * env-axis shard); exposed for drivers and for timing (class "perm").  Stream-ordered. */
int dppo_global_minibatch_lists(dppo_handle* h, const int32_t* targets, int32_t* local,
                                int32_t* seg, void* stream);

/* Multi-GPU over RCCL (xGMI): rank 0 creates the id, the caller broadcasts it (e.g. with
 * torch.distributed), every rank attaches it to its handle.  dppo_learn_f32 then all-reduces the
 * advantage statistics once and the gradient once per minibatch. */
int dppo_comm_unique_id(char* out128);
int dppo_comm_init(dppo_handle* h, int32_t nranks, int32_t rank, const char* id128);

/* Peer exchange (single node, all GPUs directly linked over xGMI): a one-shot all-reduce that
 * replaces the RCCL calls above.  Every rank exports its exchange buffer (64-byte IPC handle),
 * the caller all-gathers the handles (e.g. torch.distributed.all_gather_object) and every rank
 * opens all of them; from then on each all-reduce of dppo_learn_f32 is one kernel that publishes
 * the rank's vector in its own buffer and sums all ranks' buffers in rank order (the same bits on
 * every rank).  Works with or without a communicator (dppo_comm_init); ranks must agree on using
 * it (run dppo_peer_selftest on every rank, agree on the results, dppo_peer_close on failure).
 * Waits are bounded by DPPO_PEER_TIMEOUT_S (default 60 s); a timeout makes dppo_status return
 * DPPO_ECOMM.  No reference counterpart (the reference is single-process); replaces the
 * torch.distributed all-reduce a data-parallel wrapper of ppo.py:276-285 would issue.
 * Exchange buffers (2 MiB each) are pooled for the life of the process: dppo_destroy returns the
 * handle's buffer to the pool and the next dppo_peer_export of the same size, memory type and
 * device takes it, zeroed (round 6: a buffer allocated where freed uncached ones had been lost a
 * store).  A process uses ONE memory type (DPPO_PEER_MEM: uncached (default), fine or coarse); a
 * second type fails with DPPO_EUNSUPPORTED.  Destroy every rank's handle of an exchange group
 * before any rank exports again (a pooled buffer must not still be mapped by an old peer). */
int dppo_peer_export(dppo_handle* h, unsigned char* out64);
#define DPPO_PEER_SHARED_DEVICE 1 /* flags: some ranks share a GPU (keeps the exchange a kernel of
                                    its own instead of fusing it into the optimizer step, whose
                                    grids could not all be resident) */
int dppo_peer_open(dppo_handle* h, int32_t nranks, int32_t rank, const unsigned char* handles,
                   int32_t flags);
int dppo_peer_close(dppo_handle* h);
/* The gradient exchange of each minibatch runs inside the optimizer-step kernel (each block
 * publishes its 64 gradient sums, waits for the same block of every rank, sums in rank order,
 * then the norm and Adam as on one device): one launch after the minibatch kernel, as on one GPU.
 * The advantage statistics use the stand-alone exchange kernel.
 * every rank's `n` values summed in rank order into buf, in place (f64 != 0: doubles) */
int dppo_peer_allreduce(dppo_handle* h, void* buf, int64_t n, int32_t f64, void* stream);
/* The handle's peer exchange: out4 = {ranks (0 = none), gradient exchange fused into the
 * optimizer kernel (0/1), exchange-buffer memory (0 coarse-grained, 1 fine-grained, 2 uncached;
 * -1 = not allocated; DPPO_PEER_MEM), exchanges so far}. */
int dppo_peer_info(dppo_handle* h, int64_t* out4);
/* one exchange of a known pattern (f32 and f64) checked exactly; synchronous */
int dppo_peer_selftest(dppo_handle* h, void* stream);

/* Sticky device-side error of the handle, read WITHOUT synchronising (host-coherent word the
 * kernels write): DPPO_EHIP once a grid-wide fan-in of the single-device optimizer step timed
 * out (its workgroups were not all resident at once -- another process holding the CUs, a
 * partitioned device).  The step whose fan-in failed leaves the parameters unchanged; every later
 * call on the handle (dppo_learn_f32, dppo_get_trace, ...) returns the same error.  No reference
 * counterpart: clip_grad_norm_ + Adam (ppo.py:284-285) run as host-ordered torch ops there. */
int dppo_status(dppo_handle* h);

/* Diagnostics: `blocks` workgroups of 1024 threads, each holding `lds_bytes` of LDS, meet in the
 * same grid-wide fan-in the optimizer step uses, with a `timeout_us` bound.  A grid that fits on
 * the device completes and leaves the status OK; one that cannot be co-resident drains after the
 * timeout and sets the sticky error (dppo_status).  Stream-ordered. */
int dppo_fanin_selftest(dppo_handle* h, int32_t blocks, int32_t lds_bytes, int64_t timeout_us,
                        void* stream);

/* Single-device loopback group (parity tests of the data-parallel path without a second GPU;
 * RCCL refuses two ranks on one device): hs[r] must be rank r of world_size n (dppo_dims), all on
 * one device, n <= 8.  Their dppo_learn_f32 calls, issued concurrently from n host threads on n
 * streams, then exchange exactly what RCCL would carry (advantage statistics, per-minibatch
 * gradient + loss partials), summed in rank order on the device.  Not for production use. */
int dppo_loopback_group(dppo_handle** hs, int32_t n);

/* ---- RecurrentPPO (reference diamond/recurrent_ppo.py; the reference crashes at :78, these
 * follow its intended semantics: GRU with per-step hidden resets :82-87, the full [T, N] sequence
 * recomputed from the stored initial hidden state for every minibatch :337-341). */
typedef struct dppo_gru_handle dppo_gru_handle;

typedef struct dppo_gru_dims {
  int32_t rollout_steps; /* T */
  int32_t num_envs;      /* N */
  int32_t obs_dim;       /* D <= 32 */
  int32_t act_dim;       /* discrete actions A <= 16 */
  int32_t hidden;        /* network_hidden_dim, must be 64 */
  int32_t gru_hidden;    /* gru_hidden_dim, must be 16 */
} dppo_gru_dims;

/* One rollout as RecurrentPPO.learn stacks it (recurrent_ppo.py:306-316), device pointers. */
typedef struct dppo_gru_batch {
  const float* obs;           /* [T][N][D] */
  const int32_t* actions;     /* [T][N] */
  const float* old_log_probs; /* [T][N] cached during rollout (:219-232) */
  const float* advantages;    /* [T][N] (normalised when advantage_norm) */
  const float* returns;       /* [T][N] */
  const uint8_t* prev_dones;  /* [T][N] hidden reset before step t where set (:84) */
  const float* hx0;           /* [N][gru_hidden] hidden state at the rollout's start (:313) */
} dppo_gru_batch;

/* Flat parameter layout of RecurrentActorCriticNetwork (named_parameters() order, 16-float
 * aligned offsets; 14 tensors). */
int dppo_gru_param_layout(const dppo_gru_dims* dims, dppo_layout* out);
int dppo_gru_create(int device, const dppo_gru_dims* dims, dppo_gru_handle** out);
void dppo_gru_destroy(dppo_gru_handle* h);

/* One minibatch gradient of the recurrent PPO loss (recurrent_ppo.py:335-360): the GRU sequence
 * over all T x N samples from hx0, the clipped-surrogate + value + entropy loss on the m samples
 * idx[0..m) (flat t * N + n), divided by m_total (the global minibatch size), and the analytic
 * backward through time.  grad [layout.total + 8]: the summed gradient in the flat layout, then
 * the loss sums {policy, value, entropy} (divide by m_total).  Stream-ordered, deterministic. */
int dppo_gru_minibatch_grad_f32(dppo_gru_handle* h, const float* params,
                                const dppo_gru_batch* batch, const int32_t* idx, int32_t m,
                                int32_t m_total, const dppo_hparams* hp, float* grad,
                                void* stream);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif

#endif /* DPPO_H_ */
