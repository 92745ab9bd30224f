// libdppo C ABI: handle/workspace management and the host-side orchestration of one PPO.learn
// (reference diamond/ppo.py:224-287, continuous_ppo.py:236-299) as a stream-ordered sequence of
// gfx950 kernels, with RCCL collectives for the env-axis data-parallel case.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <thread>
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "common.h"
#include "loop_sync.h"

namespace dppo {

static thread_local char g_err[1024] = "";
thread_local LaunchTiming g_launch_timing;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

ParamOffsets offsets_from_layout(const dppo_dims& d, const dppo_layout& L) {
  ParamOffsets p{};
  const int s = d.continuous ? 1 : 0;
  p.ls = d.continuous ? L.offset[0] : -1;
  p.W1 = L.offset[s + 0];
  p.b1 = L.offset[s + 1];
  p.W2 = L.offset[s + 2];
  p.b2 = L.offset[s + 3];
  p.Wa = L.offset[s + 4];
  p.ba = L.offset[s + 5];
  p.Wo = L.offset[s + 6];
  p.bo = L.offset[s + 7];
  p.Wc = L.offset[s + 8];
  p.bc = L.offset[s + 9];
  p.Wv = L.offset[s + 10];
  p.bv = L.offset[s + 11];
  return p;
}

}  // namespace dppo

using namespace dppo;

struct dppo_handle;

// Single-device loopback group (dppo_loopback_group): n handles on ONE device, one per rank, whose
// learns are driven concurrently from n host threads on n streams.  Each all-reduce of the
// data-parallel path becomes: record "ready" on the rank's stream, host barrier, wait for every
// peer's "ready", sum the n buffers in rank order into a private scratch (rank_sum_kernel), record
// "done", host barrier, wait for every peer's "done" (nobody still reads this rank's buffer), copy
// the sum back.  RCCL refuses two ranks on one GPU; this is how the N > 1 data path
// (statistics / gradient exchange, global divisors, rank-0-only terms) is parity-tested on one.
struct LoopGroup : LoopSync {
  dppo_handle* members[kMaxLoopRanks] = {};
  void* bufs[kMaxLoopRanks] = {};
};

#define DPPO_NCCL_CHECK(expr)                                                             \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess) {                                                              \
      set_error("%s failed: %s", #expr, ncclGetErrorString(r_));                         \
      return DPPO_ECOMM;                                                                  \
    }                                                                                     \
  } while (0)

constexpr int kPermSlots = DPPO_PERM_SLOTS;
constexpr int kExtSlots = DPPO_PERM_EXT_SLOTS;

struct dppo_handle {
  int device = 0;
  dppo_dims dims{};
  dppo_layout layout{};
  ParamOffsets po{};
  MlpShape sh{};
  bool mlp_ok = false;
  int64_t B = 0;   // local samples T*N
  int32_t mb = 0;  // local minibatch size B / M
  // global-minibatch data parallelism (dims.global_minibatches with world_size > 1): the host
  // permutations cover the global batch Bg = B * world; shard_select turns them into this rank's
  // per-epoch local lists + minibatch boundaries
  bool gmb = false;
  int64_t Bg = 0;
  int64_t pe = 0;                    // permutation entries per epoch: Bg (global) or B (local)
  int32_t* perms_local = nullptr;    // [E][B]
  int32_t* seg = nullptr;            // [E][M + 1]
  int32_t* sel_cnt = nullptr;        // [E][shard_select_chunks(Bg)]
  int gae_mode = DPPO_GAE_EXACT;
  int G = 1;       // workgroups (= gradient slabs) of the fused minibatch kernel
  int num_cus = 256;
  int64_t slab_stride = 0;
  int n_partials = 0;
  // device workspace
  float *logp = nullptr, *values = nullptr, *next_values = nullptr, *adv = nullptr,
        *ret = nullptr, *adv_n = nullptr, *rec = nullptr, *slabs = nullptr, *grad = nullptr,
        *trace = nullptr, *mean_std = nullptr;
  double *partials = nullptr, *dsum = nullptr, *sq_part = nullptr;
  // next-value reuse of the old-policy evaluation (mlp.hip, EvalReuse)
  EvalReuse reuse{};
  bool reuse_on = false;
  unsigned* arrivals = nullptr;  // [4][kArrivalWords]: (unused), fused tail x 2, probe
  unsigned long long* ra_tags = nullptr;  // reduce_adam_kernel's tagged partials (optim.hip)
  // sticky device error word (grid_fanin timeouts): host-coherent pinned memory and its device
  // alias; the host reads it at the start of every call on the handle, without a sync
  unsigned* err_host = nullptr;
  unsigned* err_dev = nullptr;
  unsigned long long fanin_ticks = kFaninTimeoutTicks;
  bool radam_ok = false;  // reduce_adam_kernel's grid fits on the device at once
  unsigned fused_epoch = 0;      // launches of the fused minibatch kernel with the Adam tail
  unsigned radam_epoch = 0;      // reduce_adam launches so far on this handle (tag of the last)
  // [E][B] permutations the minibatch kernels gather with, and the Fisher-Yates targets they are
  // resolved from (dppo_learn_targets_f32); double-buffered so the next learn's upload can run
  // on the copy stream while the current learn's minibatches still read the other buffer
  int32_t* perms_dev2[2] = {nullptr, nullptr};
  int32_t* targets_dev2[2] = {nullptr, nullptr};
  int32_t* perms_dev = nullptr;     // the buffer of the learn being enqueued
  int32_t* perm_scratch = nullptr;  // Fisher-Yates resolution scratch (perm_scratch_ints)
  int64_t perm_scratch_n = 0;       // its size in int32
  int dev_slot = 0;
  hipStream_t copy_stream = nullptr;  // H2D permutation uploads, overlapped with prepare()
  hipEvent_t perms_ready = nullptr;   // upload of the current learn's permutations done
  hipEvent_t perms_free[2] = {nullptr, nullptr};  // the last learn reading device slot k is done
  bool perms_free_valid[2] = {false, false};
  // two pinned host staging slots, each with the event that marks its upload done
  // kPermSlots pinned host staging slots: one being uploaded, one ready, one being drawn
  int32_t* perms_pinned[kPermSlots] = {};
  hipEvent_t perm_copy_done[kPermSlots] = {};
  bool perm_copy_pending[kPermSlots] = {};
  // external staging slots (dppo_perm_external): caller-owned host memory, page-locked here,
  // uploaded from directly -- e.g. a node-shared draw's slots in shared memory
  int32_t* ext_ptr[kExtSlots] = {};
  int64_t ext_bytes[kExtSlots] = {};
  hipEvent_t ext_done[kExtSlots] = {};
  bool ext_pending[kExtSlots] = {};
  int32_t trace_rows = 0;
  hipStream_t last_stream = nullptr;
  hipEvent_t order_ev = nullptr;  // orders a call on another stream after the last learn
  // optional per-kernel-class timing with HIP events on the launch stream
  bool timing = false;
  struct Rec {
    int cls;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  // RCCL
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  // single-device loopback group (tests): shared by its members
  std::shared_ptr<LoopGroup> loop;
  void* loop_out = nullptr;
  size_t loop_bytes = 0;
  hipEvent_t loop_ready = nullptr, loop_done = nullptr;
  // peer exchange (peer.hip): this rank's exchange buffer, and every rank's as mapped here
  char* xbuf = nullptr;
  int64_t xbytes = 0;                // its allocation size (the process pool's key)
  int64_t xcap = 0;                  // elements (of up to 8 B) per parity
  char* xpeer[kMaxPeers] = {};
  bool xmapped[kMaxPeers] = {};      // opened with hipIpcOpenMemHandle (closed on teardown)
  int xworld = 0;                    // > 0: the exchange carries every all-reduce
  bool xfused = false;               // the gradient exchange runs inside reduce_adam_kernel
  unsigned xseq = 0;                 // exchanges so far (the same count on every rank)
  int xmem = 0;                      // exchange buffer memory: 0 coarse, 1 fine-grained, 2 uncached
  unsigned long long xticks = 0;     // wait bound of one exchange (s_memrealtime ticks)
};

namespace {

inline int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

int build_layout(const dppo_dims* d, dppo_layout* L) {
  std::memset(L, 0, sizeof(*L));
  const int H = d->hidden, D = d->obs_dim, A = d->act_dim;
  int rows[DPPO_MAX_TENSORS], cols[DPPO_MAX_TENSORS];
  int n = 0;
  auto add = [&](int r, int c) {
    rows[n] = r;
    cols[n] = c;
    ++n;
  };
  if (d->continuous) add(1, A);  // actor_log_std [1, A] (continuous_ppo.py:76), registered first
  add(H, D);                     // base.0      (ppo.py:54)
  add(H, 1);
  add(H, H);                     // base.2      (ppo.py:56)
  add(H, 1);
  add(H, H);                     // actor(_mean)_head.0 (ppo.py:61)
  add(H, 1);
  add(A, H);                     // actor(_mean)_head.2 (ppo.py:63)
  add(A, 1);
  add(H, H);                     // critic_head.0 (ppo.py:68)
  add(H, 1);
  add(1, H);                     // critic_head.2 (ppo.py:70)
  add(1, 1);
  int64_t off = 0, real = 0;
  for (int i = 0; i < n; ++i) {
    const int64_t ne = (int64_t)rows[i] * cols[i];
    L->offset[i] = off;
    L->numel[i] = ne;
    L->rows[i] = rows[i];
    L->cols[i] = cols[i];
    off = round_up(off + ne, 16);
    real += ne;
  }
  L->count = n;
  L->total = off;
  L->n_real = real;
  return DPPO_OK;
}

int validate_dims(const dppo_dims* d) {
  if (!d) {
    set_error("dims is NULL");
    return DPPO_EINVAL;
  }
  if (d->rollout_steps < 1 || d->num_envs < 1 || d->obs_dim < 1 || d->act_dim < 1 ||
      d->hidden < 1 || d->num_epochs < 1 || d->num_minibatches < 1 || d->world_size < 1 ||
      d->rank < 0 || d->rank >= d->world_size) {
    set_error("invalid dims (T=%d N=%d D=%d A=%d H=%d E=%d M=%d world=%d rank=%d)",
              d->rollout_steps, d->num_envs, d->obs_dim, d->act_dim, d->hidden, d->num_epochs,
              d->num_minibatches, d->world_size, d->rank);
    return DPPO_EINVAL;
  }
  if ((int64_t)d->rollout_steps * d->num_envs > 0x7FFFFFFF) {
    set_error("T*N exceeds int32 sample indexing");
    return DPPO_EINVAL;
  }
  return DPPO_OK;
}

// Tag of the next reduce_adam launch: never 0, the value the tag words start from.  Every launch
// rewrites every word, so after a wrap the words hold the previous launch's tag, not a stale match.
unsigned next_radam_epoch(dppo_handle* h) {
  if (++h->radam_epoch == 0u) h->radam_epoch = 1u;
  return h->radam_epoch;
}

int peer_acq();

// Test-only environment hooks (a sequence number near the 32-bit wrap, a skewed self-test
// contribution) act only with DPPO_TEST_HOOKS=1, so a stray variable cannot change a production
// run.
const char* test_hook(const char* name) {
  const char* e = std::getenv("DPPO_TEST_HOOKS");
  return e && e[0] == '1' ? std::getenv(name) : nullptr;
}

// DPPO_PEER_ACQ=1 (with DPPO_TEST_HOOKS=1; diagnosis of stale exchange-buffer reads): every poll
// of a peer word behind a system-scope acquire fence
int peer_acq() {
  static const int v = [] {
    const char* e = test_hook("DPPO_PEER_ACQ");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return v;
}

template <typename T>
int dalloc(T** p, int64_t n) {
  if (n <= 0) n = 1;
  hipError_t e = hipMalloc((void**)p, (size_t)n * sizeof(T));
  if (e != hipSuccess) {
    set_error("hipMalloc(%lld bytes) failed: %s", (long long)(n * sizeof(T)),
              hipGetErrorString(e));
    return DPPO_ENOMEM;
  }
  return DPPO_OK;
}

#define DPPO_TRY(x)       \
  do {                    \
    int rc_ = (x);        \
    if (rc_ != DPPO_OK) { \
      return rc_;         \
    }                     \
  } while (0)

inline hipStream_t S(void* s) { return (hipStream_t)s; }

// The handle's sticky device error (grid_fanin timeout), read without synchronising: a kernel
// enqueued earlier reports here once it has run -- at the latest at the first call after the
// next synchronisation (dppo_get_trace, dppo_status after a sync).
int device_status(const dppo_handle* h) {
  const unsigned e = h->err_host ? __atomic_load_n(h->err_host, __ATOMIC_ACQUIRE) : 0u;
  if (e == 0u) return DPPO_OK;
  const unsigned code = e & 0xffu, rank = (e >> 8) & 0xffu, idx = e >> 16;
  if (code == kErrPeerTimeout) {
    const unsigned seen_lo = __atomic_load_n(h->err_host + 2, __ATOMIC_ACQUIRE);
    const unsigned seen_hi = __atomic_load_n(h->err_host + 3, __ATOMIC_ACQUIRE);
    set_error("a peer exchange timed out: rank %u's word %u (slice or gradient element) did not "
              "arrive within %.0f s (DPPO_PEER_TIMEOUT_S; exchange %u, last read 0x%08x%08x) -- "
              "another rank did not reach the same all-reduce, or its publish is not visible "
              "here; that optimizer step used this rank's gradient alone and this handle is no "
              "longer usable",
              rank, idx, (double)h->xticks / 1e8, h->xseq, seen_hi, seen_lo);
    return DPPO_ECOMM;
  }
  if (code == kErrTagTimeout) {
    set_error("the optimizer step's fan-in timed out (code 3: tagged word %u never arrived at "
              "block %u -- its workgroups were not all resident at once, or a block left early); "
              "the parameters of that step were left unchanged and this handle is no longer "
              "usable", idx, rank);
    return DPPO_EHIP;
  }
  set_error("a grid-wide fan-in timed out (code %u, block %u): its workgroups were not all "
            "resident on the device at once (another process holding the CUs, or a partitioned "
            "device); the parameters of that optimizer step were left unchanged and this handle "
            "is no longer usable", code, idx);
  return DPPO_EHIP;
}

enum KClass {
  K_EVAL = 0, K_GAE, K_STATS, K_PACK, K_GRAD, K_REDUCE, K_ADAM, K_COMM, K_PERM, K_RADAM, K_PROBE,
  K_NCLASS
};

hipEvent_t pool_event(dppo_handle* h) {
  if (h->pool_used == h->pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    h->pool.push_back(e);
  }
  return h->pool[h->pool_used++];
}

// RAII bracket around the launches of one kernel class when timing is enabled.  Kernel brackets
// hand their event pair to the launches (g_launch_timing, common.h), so the events carry the
// kernels' own start/end times; `markers` brackets (RCCL calls) record the pair on the stream.
struct Timed {
  dppo_handle* h;
  hipStream_t s;
  int cls;
  bool markers;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(dppo_handle* h_, int cls_, hipStream_t s_, bool markers_ = false)
      : h(h_), s(s_), cls(cls_), markers(markers_) {
    if (!h->timing) return;
    a = pool_event(h);
    b = pool_event(h);
    if (!a || !b) {
      a = b = nullptr;
      return;
    }
    if (markers) {
      (void)hipEventRecord(a, s);
    } else {
      g_launch_timing.start = a;
      g_launch_timing.stop = b;
    }
  }
  ~Timed() {
    if (!a) return;
    if (markers) {
      (void)hipEventRecord(b, s);
    } else {
      if (g_launch_timing.start == a) {  // nothing was launched: an empty interval
        (void)hipEventRecord(a, s);
        (void)hipEventRecord(b, s);
      }
      g_launch_timing = LaunchTiming{};
    }
    h->recs.push_back({cls, a, b});
  }
};

int require_mlp(const dppo_handle* h) {
  if (!h->mlp_ok) {
    set_error("fused MLP kernels support hidden=64, obs_dim<=32, act_dim<=16 (got H=%d D=%d A=%d)",
              h->dims.hidden, h->dims.obs_dim, h->dims.act_dim);
    return DPPO_EUNSUPPORTED;
  }
  return DPPO_OK;
}

// Whether learn() takes the exchanging (multi-rank) sequence: an RCCL communicator of any size
// -- a 1-rank one too, so the collective path (slab reduce -> ncclAllReduce -> clip + Adam, the
// advantage-stat all-reduce) runs and is tested on a single GPU -- or a loopback group.
inline bool distributed(const dppo_handle* h) {
  return h->comm != nullptr || (h->loop && h->nranks > 1) || h->xworld > 0;
}
inline int world_of(const dppo_handle* h) { return distributed(h) ? h->nranks : 1; }

int loop_barrier(LoopGroup* g) {
  switch (g->barrier(std::chrono::seconds(120))) {
    case LoopSync::kOk:
      return DPPO_OK;
    case LoopSync::kTimeout:
      set_error("loopback group: a rank did not reach the all-reduce within 120 s");
      return DPPO_ECOMM;
    default:
      set_error("loopback group is broken (an exchange timed out or a member was destroyed)");
      return DPPO_ECOMM;
  }
}

int loop_allreduce(dppo_handle* h, void* buf, size_t n, bool f64, hipStream_t s) {
  LoopGroup* g = h->loop.get();
  const size_t bytes = n * (f64 ? sizeof(double) : sizeof(float));
  if (bytes > h->loop_bytes) {
    set_error("loopback all-reduce of %zu bytes exceeds the %zu-byte scratch", bytes,
              h->loop_bytes);
    return DPPO_EINVAL;
  }
  // The peers' readiness is awaited on the HOST (hipEventSynchronize), never by a device-side
  // wait on another rank's stream: with more ranks than hardware queues (GPU_MAX_HW_QUEUES)
  // streams share queues, and a cross-stream barrier packet could then wait on work queued behind
  // it.  Test-only path: two host synchronisations per exchange are fine.
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->bufs[h->rank] = buf;
  }
  DPPO_HIP_CHECK(hipEventRecord(h->loop_ready, s));
  DPPO_TRY(loop_barrier(g));
  // The peers' buffers and events are read, and their events waited for, under the group lock:
  // a peer being destroyed (dppo_destroy takes the lock to clear its slot and break the group
  // before it frees anything) then fails the exchange instead of being read after it is freed.
  // Waiting under the lock cannot deadlock: every awaited event was recorded before its rank
  // entered the barrier just passed, so it completes without any host progress.
  RankPtrs src{};
  auto wait_peers = [&](bool done) -> int {
    std::lock_guard<std::mutex> lk(g->mu);
    for (int r = 0; r < g->n; ++r) {
      if (g->broken || !g->members[r] || !g->bufs[r]) {
        set_error("loopback group is broken (a member was destroyed during an exchange)");
        return DPPO_ECOMM;
      }
      src.p[r] = g->bufs[r];
      DPPO_HIP_CHECK(
          hipEventSynchronize(done ? g->members[r]->loop_done : g->members[r]->loop_ready));
    }
    return DPPO_OK;
  };
  DPPO_TRY(wait_peers(false));
  DPPO_TRY(launch_rank_sum(src, g->n, h->loop_out, (int64_t)n, f64, s));
  DPPO_HIP_CHECK(hipEventRecord(h->loop_done, s));
  DPPO_TRY(loop_barrier(g));
  DPPO_TRY(wait_peers(true));
  DPPO_HIP_CHECK(hipMemcpyAsync(buf, h->loop_out, bytes, hipMemcpyDeviceToDevice, s));
  return DPPO_OK;
}

// Exchange numbers: the same sequence on every rank; 0 is skipped (the tagged words start as 0).
// The buffers are double-buffered by parity (seq & 1), so consecutive numbers must alternate
// parity: after 0xFFFFFFFF (odd) comes 2, not 1.
unsigned next_xseq(dppo_handle* h) {
  if (++h->xseq == 0u) h->xseq = 2u;
  return h->xseq;
}

int peer_allreduce(dppo_handle* h, void* buf, size_t n, bool f64, hipStream_t s) {
  PeerArgs a{};
  a.src = buf;
  a.dst = buf;
  for (int r = 0; r < h->xworld; ++r) a.bufs[r] = h->xpeer[r];
  a.n = (int64_t)n;
  a.data_bytes = h->xcap * 8;
  a.world = h->xworld;
  a.rank = h->rank;
  a.seq = next_xseq(h);
  a.err = h->err_dev;
  a.timeout_ticks = h->xticks;
  a.acq = peer_acq();
  return launch_peer_sum(a, f64, s);
}

int allreduce(dppo_handle* h, void* buf, size_t n, ncclDataType_t t, hipStream_t s) {
  if (!distributed(h)) return DPPO_OK;
  if (h->xworld > 0) return peer_allreduce(h, buf, n, t == ncclFloat64, s);
  if (h->loop) return loop_allreduce(h, buf, n, t == ncclFloat64, s);
  DPPO_NCCL_CHECK(ncclAllReduce(buf, buf, n, t, ncclSum, h->comm, s));
  return DPPO_OK;
}

int prepare(dppo_handle* h, const dppo_rollout* ro, const float* params, const dppo_hparams* hp,
            const dppo_learn_outputs* out, hipStream_t s) {
  DPPO_TRY(require_mlp(h));
  if (!ro || !params || !hp || !ro->obs || !ro->next_obs || !ro->actions || !ro->rewards ||
      !ro->term || !ro->trunc) {
    set_error("null rollout/params/hparams pointer");
    return DPPO_EINVAL;
  }
  const dppo_dims& d = h->dims;
  // (2) old-policy evaluation (ppo.py:235-238)
  {
    Timed tm(h, K_EVAL, s);
    DPPO_TRY(launch_eval(h->sh, h->po, params, ro->obs, ro->actions, ro->next_obs, h->logp,
                         h->values, h->next_values, h->B, s, h->reuse_on ? &h->reuse : nullptr));
  }
  // (3) GAE + returns (ppo.py:240-241)
  {
    Timed tm(h, K_GAE, s);
    DPPO_TRY(launch_gae(ro->rewards, ro->term, ro->trunc, h->values, h->next_values, h->adv,
                        h->ret, h->partials, d.rollout_steps, d.num_envs, hp->gamma,
                        hp->gae_lambda, s, &h->n_partials, h->gae_mode));
  }
  // (4) advantage statistics, global over ranks (ppo.py:243).  One rank: the pack kernel reduces
  // the GAE partials itself (one launch and one kernel boundary fewer per learn); several: the
  // reduced sums are all-reduced first.  DPPO_STATS_LAUNCH=1 keeps the separate launch (A/B).
  static const bool stats_launch = [] {
    const char* e = std::getenv("DPPO_STATS_LAUNCH");
    return e && e[0] == '1';
  }();
  // Folded only where the partials are few (the persistent GAE kernels: one per workgroup, <= the
  // CU count): every pack block re-reduces all of them, which on the fallback GAE path (N % 16 != 0
  // or unaligned buffers: one partial per 16 envs, 4,096 at N = 65,536) would be ~128 MB of
  // redundant L2 reads per learn -- there the separate reduction launch is cheaper.
  const bool fold_stats =
      hp->advantage_norm && !distributed(h) && !stats_launch && h->n_partials <= 512;
  if (hp->advantage_norm && !fold_stats) {
    {
      Timed tm(h, K_STATS, s);
      DPPO_TRY(launch_stats_reduce(h->partials, h->n_partials, h->dsum, s));
    }
    if (distributed(h)) {
      Timed tm(h, K_COMM, s, true);
      DPPO_TRY(allreduce(h, h->dsum, 2, ncclFloat64, s));
    }
  }
  // (5) sample records for the minibatch gather (ppo.py:246-249)
  PackArgs pa{};
  pa.obs = ro->obs;
  pa.actions = ro->actions;
  pa.logp = h->logp;
  pa.adv = h->adv;
  pa.ret = h->ret;
  pa.dsum = h->dsum;
  pa.partials = fold_stats ? h->partials : nullptr;
  pa.n_partials = h->n_partials;
  pa.n_total = (double)h->B * (double)world_of(h);
  pa.advantage_norm = hp->advantage_norm;
  pa.adv_out = h->adv_n;
  pa.rec = h->rec;
  pa.B = h->B;
  pa.D = d.obs_dim;
  pa.D8 = h->sh.D8;
  pa.A = d.act_dim;
  pa.R = h->sh.R;
  pa.continuous = d.continuous;
  {
    Timed tm(h, K_PACK, s);
    DPPO_TRY(launch_pack(pa, s));
  }
  if (out) {
    const size_t nb = (size_t)h->B * sizeof(float);
    if (out->log_probs)
      DPPO_HIP_CHECK(hipMemcpyAsync(out->log_probs, h->logp, nb, hipMemcpyDeviceToDevice, s));
    if (out->values)
      DPPO_HIP_CHECK(hipMemcpyAsync(out->values, h->values, nb, hipMemcpyDeviceToDevice, s));
    if (out->next_values)
      DPPO_HIP_CHECK(
          hipMemcpyAsync(out->next_values, h->next_values, nb, hipMemcpyDeviceToDevice, s));
    if (out->advantages)
      DPPO_HIP_CHECK(hipMemcpyAsync(out->advantages, h->adv_n, nb, hipMemcpyDeviceToDevice, s));
    if (out->returns)
      DPPO_HIP_CHECK(hipMemcpyAsync(out->returns, h->ret, nb, hipMemcpyDeviceToDevice, s));
  }
  return DPPO_OK;
}

// One minibatch: fused gradient kernel -> slab reduction -> [all-reduce] (grad left in h->grad).
int minibatch_grad(dppo_handle* h, const float* params, const int32_t* idx, const int32_t* seg,
                   int32_t m, int32_t m_total, const dppo_hparams* hp, hipStream_t s) {
  const dppo_dims& d = h->dims;
  GradArgs ga{};
  ga.params = params;
  ga.rec = h->rec;
  ga.idx = idx;
  ga.seg = seg;
  ga.m = m;
  ga.inv_m = (float)(1.0 / (double)m_total);
  ga.clip_eps = hp->ppo_clip;
  ga.vf_coef = hp->value_loss_weight;
  ga.ent_coef = hp->entropy_beta;
  ga.slabs = h->slabs;
  ga.slab_stride = h->slab_stride;
  ga.p_total = h->layout.total;
  // with `seg` the size is known only on the device: the handle's grid (sized for the largest
  // share a rank can hold) -- workgroups past the last step contribute zero slabs
  int G = seg ? h->G : mb_grid(h->sh, m);
  if (G > h->G) G = h->G;
  {
    Timed tm(h, K_GRAD, s);
    DPPO_TRY(launch_mb(h->sh, h->po, ga, G, s));
  }
  {
    Timed tm(h, K_REDUCE, s);
    DPPO_TRY(launch_slab_reduce(h->slabs, G, h->slab_stride, h->layout.total, h->grad, h->sq_part,
                                h->po.ls, d.continuous ? d.act_dim : 0, hp->entropy_beta,
                                (d.continuous && h->rank == 0) ? 1 : 0, s));
  }
  if (distributed(h)) {
    Timed tm(h, K_COMM, s, true);
    DPPO_TRY(allreduce(h, h->grad, (size_t)h->layout.total + 8, ncclFloat32, s));
  }
  return DPPO_OK;
}

}  // namespace

namespace {

// Upload the host [E][B] buffer (permutations or Fisher-Yates targets) into device buffer `dst`
// (device slot `ds`) on the handle's copy stream, so the PCIe transfer (8 MB at B = 524,288) runs
// beside the old-policy eval / GAE / pack kernels instead of in front of them.  The copy first
// waits for the previous learn that read device slot `ds`; `perms_ready` marks the upload done
// and the launch stream waits on it before the first kernel that reads the permutations.  A
// pinned slot is copied from directly (pure DMA); any other buffer is first staged in slot 0.
int upload_perms(dppo_handle* h, const int32_t* host, int32_t* dst, int ds) {
  const size_t pbytes = (size_t)(h->dims.num_epochs * h->pe) * sizeof(int32_t);
  for (int k = 0; k < kExtSlots; ++k) {
    if (!h->ext_ptr[k] || host != h->ext_ptr[k]) continue;
    if ((int64_t)pbytes > h->ext_bytes[k]) {
      set_error("external permutation slot %d holds %lld bytes, the learn needs %zu", k,
                (long long)h->ext_bytes[k], pbytes);
      return DPPO_EINVAL;
    }
    if (h->perms_free_valid[ds])
      DPPO_HIP_CHECK(hipStreamWaitEvent(h->copy_stream, h->perms_free[ds], 0));
    DPPO_HIP_CHECK(hipMemcpyAsync(dst, host, pbytes, hipMemcpyHostToDevice, h->copy_stream));
    DPPO_HIP_CHECK(hipEventRecord(h->ext_done[k], h->copy_stream));
    DPPO_HIP_CHECK(hipEventRecord(h->perms_ready, h->copy_stream));
    h->ext_pending[k] = true;
    return DPPO_OK;
  }
  int slot = 0;
  for (int k = 1; k < kPermSlots; ++k)
    if (host == h->perms_pinned[k]) slot = k;
  if (host != h->perms_pinned[slot]) {
    if (h->perm_copy_pending[0]) DPPO_HIP_CHECK(hipEventSynchronize(h->perm_copy_done[0]));
    std::memcpy(h->perms_pinned[0], host, pbytes);
  }
  if (h->perms_free_valid[ds])
    DPPO_HIP_CHECK(hipStreamWaitEvent(h->copy_stream, h->perms_free[ds], 0));
  DPPO_HIP_CHECK(hipMemcpyAsync(dst, h->perms_pinned[slot], pbytes, hipMemcpyHostToDevice,
                                h->copy_stream));
  DPPO_HIP_CHECK(hipEventRecord(h->perm_copy_done[slot], h->copy_stream));
  DPPO_HIP_CHECK(hipEventRecord(h->perms_ready, h->copy_stream));
  h->perm_copy_pending[slot] = true;
  return DPPO_OK;
}

// Calls that use the handle's workspace run after the previous such call even when the caller
// switches streams (one extra event record + wait only then); the stream becomes the one the
// next call follows.
int order_after_last(dppo_handle* h, hipStream_t s) {
  if (h->last_stream && h->last_stream != s) {
    if (!h->order_ev) DPPO_HIP_CHECK(hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming));
    DPPO_HIP_CHECK(hipEventRecord(h->order_ev, h->last_stream));
    DPPO_HIP_CHECK(hipStreamWaitEvent(s, h->order_ev, 0));
  }
  h->last_stream = s;
  return DPPO_OK;
}

int learn_impl(dppo_handle* h, const dppo_rollout* rollout, float* params, float* adam_m,
               float* adam_v, const dppo_hparams* hp, const int32_t* host_buf, bool targets,
               const dppo_learn_outputs* outputs, void* stream) {
  if (!h || !params || !adam_m || !adam_v || !hp || !host_buf) {
    set_error("null argument to dppo_learn_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  const dppo_dims& d = h->dims;
  if (h->pe % d.num_minibatches != 0) {
    // the reference's perms.reshape(E, M, B // M) raises ValueError (ppo.py:255)
    set_error("cannot reshape array of size %lld into shape (%d,%d,%lld)",
              (long long)(h->pe * d.num_epochs), d.num_epochs, d.num_minibatches,
              (long long)(h->pe / d.num_minibatches));
    return DPPO_EINVAL;
  }
  if (h->gmb && !(distributed(h) && h->nranks == d.world_size)) {
    set_error("global_minibatches needs the world_size=%d communicator (dppo_comm_init or "
              "dppo_loopback_group) before dppo_learn_f32", d.world_size);
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t s = S(stream);
  DPPO_TRY(order_after_last(h, s));
  const int64_t E = d.num_epochs, M = d.num_minibatches;
  // permutations (ppo.py:252-255): host -> pinned staging -> device on the copy stream, beside
  // prepare(); given as swap targets they are shuffled on the device after prepare()
  const int ds = h->dev_slot;
  h->dev_slot ^= 1;
  h->perms_dev = h->perms_dev2[ds];
  DPPO_TRY(upload_perms(h, host_buf, targets ? h->targets_dev2[ds] : h->perms_dev, ds));
  DPPO_TRY(prepare(h, rollout, params, hp, outputs, s));
  DPPO_HIP_CHECK(hipStreamWaitEvent(s, h->perms_ready, 0));
  if (targets && h->gmb && perm_walk()) {
    // global minibatches from the swap targets: only this rank's samples are walked to their
    // positions (the whole permutation is never resolved; perms_dev holds the marks)
    Timed tm(h, K_PERM, s);
    DPPO_TRY(launch_shard_select_targets(h->targets_dev2[ds], h->perms_dev, h->perm_scratch,
                                         h->perm_scratch_n, h->perms_local, h->seg, h->sel_cnt, h->Bg,
                                         d.num_envs * h->nranks, d.num_envs * h->rank,
                                         d.num_envs, (int32_t)E, (int32_t)M, s));
  } else if (targets) {
    Timed tm(h, K_PERM, s);
    DPPO_TRY(launch_perm_resolve(h->targets_dev2[ds], h->perms_dev, h->pe, (int32_t)E,
                                 h->perm_scratch, h->perm_scratch_n, s));
  }
  if (h->gmb && !(targets && perm_walk())) {
    // this rank's members of every global minibatch, in permutation order
    Timed tm(h, K_PERM, s);
    DPPO_TRY(launch_shard_select(h->perms_dev, h->perms_local, h->seg, h->sel_cnt, h->Bg,
                                 d.num_envs * h->nranks, d.num_envs * h->rank, d.num_envs,
                                 (int32_t)E, (int32_t)M, s));
  }
  // (6) E x M dependent optimizer steps (ppo.py:258-285)
  const int32_t mb = h->mb;
  // global minibatch size: the divisor of every mean (ppo.py:270-274)
  const int32_t m_total = h->gmb ? (int32_t)(h->Bg / M) : mb * world_of(h);
  const float inv_m = (float)(1.0 / (double)m_total);
  for (int64_t e = 0; e < E; ++e) {
    for (int64_t j = 0; j < M; ++j) {
      const int64_t k = e * M + j;
      const int32_t* idx =
          h->gmb ? h->perms_local + e * h->B : h->perms_dev + e * h->B + j * mb;
      const int32_t* seg = h->gmb ? h->seg + e * (M + 1) + j : nullptr;
      const double step = (double)(hp->adam_step + k + 1);
      const double bc1 = 1.0 - std::pow((double)hp->adam_beta1, step);
      const double bc2 = 1.0 - std::pow((double)hp->adam_beta2, step);
      const double step_size = hp->lr / bc1;
      const double bc2_sqrt = std::pow(bc2, 0.5);
      float* trace = h->trace + k * DPPO_TRACE_FIELDS;
      // DPPO_SPLIT_ADAM=1 (parity tests): the multi-rank sequence -- minibatch kernel, slab
      // reduction, [all-reduce], clip + Adam kernel -- on one device, so the N > 1 kernels are
      // checked against the reference traces without a second GPU
      // A device that cannot hold reduce_adam_kernel's grid at once takes the same sequence.
      // Over a peer exchange the cross-rank sum runs inside reduce_adam_kernel (each block
      // publishes its slice and sums the ranks' slices before the norm), so the multi-rank learn
      // keeps the single-device sequence: minibatch kernel -> reduce_adam, one launch each.
      const bool split = std::getenv("DPPO_SPLIT_ADAM") != nullptr;
      const bool peer = h->xworld > 0 && h->xfused && h->radam_ok && !split;
      const bool multi = (distributed(h) && !peer) || !h->radam_ok || split;
      if (!multi) {
        // single device (or peer exchange): fused kernel -> slab reduce + clip + Adam in one launch
        GradArgs ga{};
        ga.params = params;
        ga.rec = h->rec;
        ga.idx = idx;
        ga.seg = seg;
        ga.m = mb;
        ga.inv_m = inv_m;
        ga.clip_eps = hp->ppo_clip;
        ga.vf_coef = hp->value_loss_weight;
        ga.ent_coef = hp->entropy_beta;
        ga.slabs = h->slabs;
        ga.slab_stride = h->slab_stride;
        ga.p_total = h->layout.total;
        const bool fused_tail = std::getenv("DPPO_FUSED_ADAM") != nullptr && !peer;
        // with `seg` (global minibatches) the share is known only on the device: the handle's
        // grid, as minibatch_grad
        int G = seg ? h->G : mb_grid(h->sh, mb, fused_tail);
        if (G > h->G) G = h->G;
        // DPPO_FUSED_ADAM=1: the slab reduction, clip and Adam as the minibatch kernel's own
        // tail (one launch per minibatch, two grid fan-ins).  Measured: the tail costs what
        // reduce_adam_kernel does (~8 us: the fan-ins, not the launch, dominate), throughput
        // within ~1.5 %; the separate kernel stays the default (and keeps the minibatch kernel's
        // roofline its own).
        if (fused_tail) {
          FusedAdam fa{};
          fa.grad = h->grad;
          fa.sq_part = h->sq_part;
          fa.arrivals = h->arrivals + kArrivalWords;
          fa.epoch = ++h->fused_epoch;
          fa.err = h->err_dev;
          fa.timeout_ticks = h->fanin_ticks;
          fa.params = params;
          fa.m = adam_m;
          fa.v = adam_v;
          fa.max_norm = hp->grad_norm_clip;
          fa.neg_step_size = (float)(-step_size);
          fa.bc2_sqrt = (float)bc2_sqrt;
          fa.beta1 = hp->adam_beta1;
          fa.beta2 = hp->adam_beta2;
          fa.eps = hp->adam_eps;
          fa.trace = trace;
          fa.ls_off = h->po.ls;
          fa.ls_n = d.continuous ? d.act_dim : 0;
          fa.add_entropy_const = d.continuous ? 1 : 0;
          Timed tm(h, K_GRAD, s);
          DPPO_TRY(launch_mb(h->sh, h->po, ga, G, s, &fa));
          continue;
        }
        {
          Timed tm(h, K_GRAD, s);
          DPPO_TRY(launch_mb(h->sh, h->po, ga, G, s));
        }
        Timed tm(h, K_RADAM, s);
#ifdef DPPO_ABL_RADAM_G1
        const int Gr = 1;  // timing-only ablation: the fixed cost of the launch without slab reads
#elif defined(DPPO_ABL_HALF_SLABS)
        const int Gr = (G + 1) / 2;  // timing-only: half the slab bytes (mbwave.hip ablation)
#else
        const int Gr = G;
#endif
        PeerArgs pa{};
        if (peer) {
          for (int r = 0; r < h->xworld; ++r) pa.bufs[r] = h->xpeer[r];
          pa.data_bytes = h->xcap * 8;
          pa.world = h->xworld;
          pa.rank = h->rank;
          pa.seq = next_xseq(h);
          pa.err = h->err_dev;
          pa.timeout_ticks = h->xticks;
          pa.acq = peer_acq();
        }
        // a block's intra-device fan-in starts after its peer wait: bound it like the peer wait
        const unsigned long long fan_ticks =
            peer && h->xticks > h->fanin_ticks ? h->xticks : h->fanin_ticks;
        DPPO_TRY(launch_reduce_adam(
            h->slabs, Gr, h->slab_stride, h->layout.total, h->grad, h->ra_tags, h->po.ls,
            d.continuous ? d.act_dim : 0, hp->entropy_beta,
            (d.continuous && h->rank == 0) ? 1 : 0, next_radam_epoch(h), params, adam_m,
            adam_v, hp->grad_norm_clip, (float)(-step_size), (float)bc2_sqrt,
            hp->adam_beta1, hp->adam_beta2, hp->adam_eps, trace, inv_m, hp->value_loss_weight,
            hp->entropy_beta, h->err_dev, fan_ticks, s, peer ? &pa : nullptr));
        continue;
      }
      DPPO_TRY(minibatch_grad(h, params, idx, seg, mb, m_total, hp, s));
      Timed tm(h, K_ADAM, s);
      // after the all-reduce the reduce kernel's per-block norm partials are stale: the Adam
      // kernel recomputes the norm from the gradient itself (every block, in one fixed order;
      // measured cheaper than the grid fan-in of reduce_adam_kernel over the reduced gradient)
      DPPO_TRY(launch_clip_adam_traced(params, h->grad, adam_m, adam_v, h->layout.total, nullptr,
                                       slab_reduce_blocks(h->layout.total), hp->grad_norm_clip,
                                       (float)(-step_size), (float)bc2_sqrt, hp->adam_beta1,
                                       hp->adam_beta2, hp->adam_eps, nullptr, trace, inv_m,
                                       hp->value_loss_weight, hp->entropy_beta, s));
    }
  }
  // device slot ds may be overwritten by an upload once this learn's minibatches are done
  DPPO_HIP_CHECK(hipEventRecord(h->perms_free[ds], s));
  h->perms_free_valid[ds] = true;
  h->last_stream = s;
  return DPPO_OK;
}

}  // namespace

extern "C" {

const char* dppo_version(void) { return "libdppo 0.1.0 (gfx950)"; }

const char* dppo_last_error(void) { return g_err; }

int dppo_param_layout(const dppo_dims* dims, dppo_layout* out) {
  DPPO_TRY(validate_dims(dims));
  if (!out) {
    set_error("out is NULL");
    return DPPO_EINVAL;
  }
  return build_layout(dims, out);
}

int dppo_create(int device, const dppo_dims* dims, dppo_handle** out) {
  DPPO_TRY(validate_dims(dims));
  if (!out) {
    set_error("out is NULL");
    return DPPO_EINVAL;
  }
  *out = nullptr;
  DPPO_HIP_CHECK(hipSetDevice(device));
  dppo_handle* h = new dppo_handle();
  h->device = device;
  h->dims = *dims;
  build_layout(dims, &h->layout);
  h->po = offsets_from_layout(*dims, h->layout);
  h->B = (int64_t)dims->rollout_steps * dims->num_envs;
  h->mb = (int32_t)(h->B / dims->num_minibatches);
  h->rank = dims->rank;
  h->nranks = dims->world_size;
  h->gmb = dims->global_minibatches != 0 && dims->world_size > 1;
  h->Bg = h->B * dims->world_size;
  h->pe = h->gmb ? h->Bg : h->B;
  const int D8 = (dims->obs_dim + 7) / 8 * 8;
  h->sh.D = dims->obs_dim;
  h->sh.D8 = D8;
  h->sh.A = dims->act_dim;
  h->sh.continuous = dims->continuous;
  h->sh.R = D8 + 4 + (dims->continuous ? (dims->act_dim + 3) / 4 * 4 : 0);
  h->mlp_ok = dims->hidden == 64 && dims->obs_dim <= 32 && dims->act_dim <= 16 &&
              mb_lds_bytes(h->sh) <= 160 * 1024 &&
              (size_t)(h->layout.total + 8) * 4 <= 160 * 1024;
  // One fused-minibatch workgroup per CU (its LDS footprint admits exactly one): never launch
  // more workgroups than CUs, or the surplus runs as a second, serialised round.
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus <= 0)
    cus = 256;
  h->num_cus = cus;
  // global minibatches: a rank's share of one varies around mb; size the grid for a whole one
  // (the larger of the two kernels' grids: DPPO_FUSED_ADAM runs the two-team kernel)
  {
    const int32_t mg = h->gmb ? (int32_t)std::min<int64_t>(h->Bg / dims->num_minibatches, h->B)
                              : (h->mb > 0 ? h->mb : 1);
    h->G = std::max(mb_grid(h->sh, mg), mb_grid(h->sh, mg, true));
  }
  if (h->G > cus) h->G = cus;
  h->slab_stride = round_up(h->layout.total + 8, 64);
  const int64_t E = dims->num_epochs, M = dims->num_minibatches;
  h->trace_rows = (int32_t)(E * M);
  int rc = DPPO_OK;
  auto chk = [&](int r) {
    if (rc == DPPO_OK && r != DPPO_OK) rc = r;
  };
  chk(dalloc(&h->logp, h->B));
  chk(dalloc(&h->values, h->B));
  chk(dalloc(&h->next_values, h->B));
  chk(dalloc(&h->adv, h->B));
  chk(dalloc(&h->ret, h->B));
  chk(dalloc(&h->adv_n, h->B));
  chk(dalloc(&h->rec, h->B * h->sh.R));
  chk(dalloc(&h->slabs, (int64_t)h->G * h->slab_stride));
  chk(dalloc(&h->grad, h->slab_stride));
  chk(dalloc(&h->trace, E * M * DPPO_TRACE_FIELDS));
  chk(dalloc(&h->mean_std, 4));
  chk(dalloc(&h->partials, 2 * ((int64_t)(dims->num_envs + 15) / 16 + 1)));
  chk(dalloc(&h->dsum, 4));
  chk(dalloc(&h->sq_part, slab_reduce_blocks(h->layout.total)));
  chk(dalloc(&h->arrivals, 4 * kArrivalWords));
  chk(dalloc(&h->ra_tags, reduce_adam_tag_words(h->layout.total)));
  {
    // DPPO_EVAL_REUSE=0: the full next_obs critic pass (A/B runs)
    const char* e = std::getenv("DPPO_EVAL_REUSE");
    h->reuse_on = dims->rollout_steps >= 2 && !(e && e[0] == '0');
    if (h->reuse_on) h->reuse.row = dims->num_envs;
  }
  for (int k = 0; k < 2; ++k) {
    chk(dalloc(&h->perms_dev2[k], E * h->pe));
    chk(dalloc(&h->targets_dev2[k], E * h->pe));
  }
  h->perms_dev = h->perms_dev2[0];
  h->perm_scratch_n = perm_scratch_ints(h->pe, (int32_t)E);
  chk(dalloc(&h->perm_scratch, h->perm_scratch_n));
  if (h->gmb) {
    chk(dalloc(&h->perms_local, E * h->B));
    chk(dalloc(&h->seg, E * (M + 1)));
    chk(dalloc(&h->sel_cnt, E * shard_select_chunks(h->Bg)));
  }
  if (rc == DPPO_OK) {
    if (hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->perms_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->perms_free[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->perms_free[1], hipEventDisableTiming) != hipSuccess) {
      set_error("hipStreamCreate / hipEventCreate failed");
      rc = DPPO_EHIP;
    }
  }
  if (rc == DPPO_OK) {
    if (hipHostMalloc((void**)&h->err_host, 64, hipHostMallocCoherent | hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&h->err_dev, h->err_host, 0) != hipSuccess) {
      set_error("hipHostMalloc (coherent error word) failed");
      rc = DPPO_EHIP;
    } else {
      for (int k = 15; k >= 0; --k) __atomic_store_n(h->err_host + k, 0u, __ATOMIC_RELEASE);
    }
  }
  // The single-device optimizer step waits in a grid-wide fan-in: take it only when its whole
  // grid fits on the device at once (a partitioned device or an occupancy surprise takes the
  // three-kernel path -- slab reduce, clip + Adam -- instead, which needs no co-residency).
  h->radam_ok =
      reduce_adam_capacity(device, h->layout.total) >= reduce_adam_blocks(h->layout.total);
  for (int k = 0; k < kPermSlots && rc == DPPO_OK; ++k) {
    hipError_t e = hipHostMalloc((void**)&h->perms_pinned[k],
                                 (size_t)(E * h->pe) * sizeof(int32_t), hipHostMallocDefault);
    if (e != hipSuccess) {
      set_error("hipHostMalloc failed: %s", hipGetErrorString(e));
      rc = DPPO_ENOMEM;
    } else if (hipEventCreateWithFlags(&h->perm_copy_done[k], hipEventDisableTiming) !=
               hipSuccess) {
      set_error("hipEventCreate failed");
      rc = DPPO_EHIP;
    }
  }
  if (rc == DPPO_OK) {
    (void)hipMemset(h->trace, 0, (size_t)E * M * DPPO_TRACE_FIELDS * sizeof(float));
    (void)hipMemset(h->dsum, 0, 4 * sizeof(double));
    (void)hipMemset(h->arrivals, 0, 4 * kArrivalWords * sizeof(unsigned));
    (void)hipMemset(h->ra_tags, 0, reduce_adam_tag_words(h->layout.total) * sizeof(uint64_t));
    // the fused kernel never writes the layout's padding floats: keep them zero in every slab
    (void)hipMemset(h->slabs, 0, (size_t)h->G * h->slab_stride * sizeof(float));
  }
  if (rc != DPPO_OK) {
    dppo_destroy(h);
    return rc;
  }
  *out = h;
  return DPPO_OK;
}

static void xpool_put(dppo_handle* h);  // (peer exchange section below)

void dppo_destroy(dppo_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  if (h->loop) {  // peers must never touch this handle's events or buffers again
    std::lock_guard<std::mutex> lk(h->loop->mu);
    h->loop->members[h->rank] = nullptr;
    h->loop->bufs[h->rank] = nullptr;
    h->loop->break_locked();
  }
  if (h->comm) ncclCommDestroy(h->comm);
  for (int r = 0; r < kMaxPeers; ++r)
    if (h->xmapped[r]) (void)hipIpcCloseMemHandle(h->xpeer[r]);
  xpool_put(h);  // kept for the next handle, never freed (peer_export)
  if (h->loop_out) (void)hipFree(h->loop_out);
  if (h->loop_ready) (void)hipEventDestroy(h->loop_ready);
  if (h->loop_done) (void)hipEventDestroy(h->loop_done);
  (void)hipFree(h->logp);
  (void)hipFree(h->values);
  (void)hipFree(h->next_values);
  (void)hipFree(h->adv);
  (void)hipFree(h->ret);
  (void)hipFree(h->adv_n);
  (void)hipFree(h->rec);
  (void)hipFree(h->slabs);
  (void)hipFree(h->grad);
  (void)hipFree(h->trace);
  (void)hipFree(h->mean_std);
  (void)hipFree(h->partials);
  (void)hipFree(h->dsum);
  (void)hipFree(h->sq_part);
  (void)hipFree(h->arrivals);
  (void)hipFree(h->ra_tags);
  for (int k = 0; k < 2; ++k) {
    (void)hipFree(h->perms_dev2[k]);
    (void)hipFree(h->targets_dev2[k]);
    if (h->perms_free[k]) (void)hipEventDestroy(h->perms_free[k]);
  }
  if (h->perms_ready) (void)hipEventDestroy(h->perms_ready);
  if (h->order_ev) (void)hipEventDestroy(h->order_ev);
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  (void)hipFree(h->perm_scratch);
  (void)hipFree(h->perms_local);
  (void)hipFree(h->seg);
  (void)hipFree(h->sel_cnt);
  for (int k = 0; k < kPermSlots; ++k) {
    if (h->perms_pinned[k]) (void)hipHostFree(h->perms_pinned[k]);
    if (h->perm_copy_done[k]) (void)hipEventDestroy(h->perm_copy_done[k]);
  }
  for (int k = 0; k < kExtSlots; ++k) {
    if (h->ext_ptr[k]) (void)hipHostUnregister(h->ext_ptr[k]);
    if (h->ext_done[k]) (void)hipEventDestroy(h->ext_done[k]);
  }
  for (hipEvent_t e : h->pool) (void)hipEventDestroy(e);
  if (h->err_host) (void)hipHostFree(h->err_host);
  delete h;
}

int dppo_gae_f32(dppo_handle* h, const float* rewards, const uint8_t* term, const uint8_t* trunc,
                 const float* values, const float* next_values, float* adv, float* returns,
                 float gamma, float gae_lambda, void* stream) {
  if (!h || !rewards || !term || !trunc || !values || !next_values || !adv || !returns) {
    set_error("null argument to dppo_gae_f32");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  Timed tm(h, K_GAE, S(stream));
  return launch_gae(rewards, term, trunc, values, next_values, adv, returns, h->partials,
                    h->dims.rollout_steps, h->dims.num_envs, gamma, gae_lambda, S(stream),
                    &h->n_partials, h->gae_mode);
}

int dppo_gae_stream_probe(dppo_handle* h, const float* rewards, const uint8_t* term,
                          const uint8_t* trunc, const float* values, const float* next_values,
                          float* adv, float* returns, void* stream) {
  if (!h || !rewards || !term || !trunc || !values || !next_values || !adv || !returns) {
    set_error("null argument to dppo_gae_stream_probe");
    return DPPO_EINVAL;
  }
  const int64_t n = (int64_t)h->dims.rollout_steps * h->dims.num_envs;
  const uintptr_t al = (uintptr_t)rewards | (uintptr_t)values | (uintptr_t)next_values |
                       (uintptr_t)adv | (uintptr_t)returns | (uintptr_t)term | (uintptr_t)trunc;
  if (n % 4 != 0 || al % 16 != 0) {
    set_error("dppo_gae_stream_probe: T*N must be a multiple of 4 and every buffer 16-B aligned");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  Timed tm(h, K_PROBE, S(stream));
  return launch_gae_stream_probe(rewards, term, trunc, values, next_values, adv, returns, n,
                                 S(stream));
}

int dppo_set_gae_mode(dppo_handle* h, int32_t mode) {
  if (!h || (mode != DPPO_GAE_EXACT && mode != DPPO_GAE_AFFINE)) {
    set_error("invalid argument to dppo_set_gae_mode");
    return DPPO_EINVAL;
  }
  h->gae_mode = mode;
  return DPPO_OK;
}

int dppo_adv_stats(dppo_handle* h, float* mean_std, void* stream) {
  if (!h || !mean_std) {
    set_error("null argument to dppo_adv_stats");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  DPPO_TRY(launch_stats_reduce(h->partials, h->n_partials, h->dsum, S(stream)));
  DPPO_TRY(allreduce(h, h->dsum, 2, ncclFloat64, S(stream)));
  const double n = (double)h->B * (double)world_of(h);
  return launch_stats_finalize(h->dsum, n, mean_std, S(stream));
}

int dppo_adv_sums(dppo_handle* h, double* sums, void* stream) {
  if (!h || !sums) {
    set_error("null argument to dppo_adv_sums");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  DPPO_TRY(launch_stats_reduce(h->partials, h->n_partials, h->dsum, S(stream)));
  DPPO_HIP_CHECK(hipMemcpyAsync(sums, h->dsum, 2 * sizeof(double), hipMemcpyDeviceToDevice,
                                S(stream)));
  return DPPO_OK;
}

int dppo_adv_stats_from_sums(const double* sums, double n_total, float* mean_std, void* stream) {
  if (!sums || !mean_std || !(n_total >= 1.0)) {
    set_error("invalid argument to dppo_adv_stats_from_sums");
    return DPPO_EINVAL;
  }
  return launch_stats_finalize(sums, n_total, mean_std, S(stream));
}

int dppo_adv_normalize_f32(float* adv, const float* mean_std, int64_t n, void* stream) {
  if (!adv || !mean_std || n < 0) {
    set_error("invalid argument to dppo_adv_normalize_f32");
    return DPPO_EINVAL;
  }
  return launch_adv_normalize(adv, mean_std, n, S(stream));
}

int dppo_old_policy_f32(dppo_handle* h, const float* params, const float* obs, const void* actions,
                        const float* next_obs, float* log_probs, float* values, float* next_values,
                        int64_t n, void* stream) {
  if (!h || !params || !obs || !actions || !next_obs || !log_probs || !values || !next_values ||
      n < 0) {
    set_error("invalid argument to dppo_old_policy_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(require_mlp(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  Timed tm(h, K_EVAL, S(stream));
  return launch_eval(h->sh, h->po, params, obs, actions, next_obs, log_probs, values,
                     next_values, n, S(stream));
}

int dppo_act_f32(dppo_handle* h, const float* params, const float* obs, int64_t n, uint64_t seed,
                 uint64_t counter, void* actions, void* stream) {
  if (!h || !params || !obs || !actions || n < 0) {
    set_error("invalid argument to dppo_act_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(require_mlp(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  return launch_act(h->sh, h->po, params, obs, actions, n, seed, counter, S(stream));
}

int dppo_act_squash_f32(dppo_handle* h, const float* params, const float* obs, int64_t n,
                        uint64_t seed, uint64_t counter, const float* low, const float* high,
                        float* actions, float* env_actions, void* stream) {
  if (!h || !params || !obs || !actions || !env_actions || n < 0 || (!low) != (!high)) {
    set_error("invalid argument to dppo_act_squash_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(require_mlp(h));
  if (!h->dims.continuous) {
    set_error("dppo_act_squash_f32 needs a continuous (Box) action space");
    return DPPO_EINVAL;
  }
  if (low) {
    for (int j = 0; j < h->dims.act_dim; ++j) {
      if (!std::isfinite(low[j]) || !std::isfinite(high[j]) || !(high[j] > low[j])) {
        set_error("dppo_act_squash_f32: bounds must be finite with high > low (dim %d)", j);
        return DPPO_EINVAL;
      }
    }
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  const ActSquash sq{env_actions, low, high};
  return launch_act(h->sh, h->po, params, obs, actions, n, seed, counter, S(stream), nullptr, &sq);
}

int dppo_actor_forward_f32(dppo_handle* h, const float* params, const float* obs, int64_t n,
                           float* heads, void* stream) {
  if (!h || !params || !obs || !heads || n < 0) {
    set_error("invalid argument to dppo_actor_forward_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(require_mlp(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  return launch_act(h->sh, h->po, params, obs, nullptr, n, 0, 0, S(stream), heads);
}

int dppo_prepare_f32(dppo_handle* h, const dppo_rollout* rollout, const float* params,
                     const dppo_hparams* hp, const dppo_learn_outputs* outputs, void* stream) {
  if (!h) {
    set_error("null handle");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  return prepare(h, rollout, params, hp, outputs, S(stream));
}

int dppo_status(dppo_handle* h) {
  if (!h) {
    set_error("null handle");
    return DPPO_EINVAL;
  }
  return device_status(h);
}

int dppo_fanin_selftest(dppo_handle* h, int32_t blocks, int32_t lds_bytes, int64_t timeout_us,
                        void* stream) {
  if (!h || blocks < 1 || lds_bytes < 0 || lds_bytes > 160 * 1024 || timeout_us < 1) {
    set_error("invalid argument to dppo_fanin_selftest");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t s = S(stream);
  unsigned* ctr = h->arrivals + 3 * kArrivalWords;  // fresh counters: this grid size, epoch 1
  DPPO_HIP_CHECK(hipMemsetAsync(ctr, 0, kArrivalWords * sizeof(unsigned), s));
  return launch_fanin_probe(blocks, lds_bytes, ctr, h->err_dev,
                            (unsigned long long)timeout_us * 100ull, s);
}

int dppo_minibatch_grad_f32(dppo_handle* h, const float* params, const int32_t* idx, int32_t m,
                            int32_t m_total, const dppo_hparams* hp, float* grad, float* loss4,
                            void* stream) {
  if (!h || !params || !idx || !hp || !grad || m < 0 || m_total <= 0) {
    set_error("invalid argument to dppo_minibatch_grad_f32");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  DPPO_TRY(require_mlp(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t s = S(stream);
  DPPO_TRY(minibatch_grad(h, params, idx, nullptr, m, m_total, hp, s));
  DPPO_HIP_CHECK(hipMemcpyAsync(grad, h->grad, (size_t)h->layout.total * sizeof(float),
                                hipMemcpyDeviceToDevice, s));
  if (loss4) {
    // {loss, loss_policy, loss_value, entropy} from the summed per-sample terms (host output)
    float tmp[8];
    DPPO_HIP_CHECK(hipMemcpyAsync(tmp, h->grad + h->layout.total, 8 * sizeof(float),
                                  hipMemcpyDeviceToHost, s));
    DPPO_HIP_CHECK(hipStreamSynchronize(s));
    const float inv = (float)(1.0 / (double)m_total);
    const float lpi = tmp[0] * inv, lv = tmp[1] * inv, ent = tmp[2] * inv;
    loss4[0] = lpi + hp->value_loss_weight * lv - hp->entropy_beta * ent;
    loss4[1] = lpi;
    loss4[2] = lv;
    loss4[3] = ent;
  }
  return DPPO_OK;
}

int dppo_clip_adam_f32(float* params, float* grad, float* adam_m, float* adam_v, int64_t n,
                       float max_norm, double lr, float beta1, float beta2, float eps, int64_t step,
                       float* out_norm, void* stream) {
  if (!params || !grad || !adam_m || !adam_v || n < 0 || step < 1) {
    set_error("invalid argument to dppo_clip_adam_f32");
    return DPPO_EINVAL;
  }
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const double step_size = lr / bc1;
  const double bc2_sqrt = std::pow(bc2, 0.5);
  return launch_clip_adam(params, grad, adam_m, adam_v, n, max_norm, (float)(-step_size),
                          (float)bc2_sqrt, beta1, beta2, eps, out_norm, S(stream));
}


int dppo_learn_f32(dppo_handle* h, const dppo_rollout* rollout, float* params, float* adam_m,
                   float* adam_v, const dppo_hparams* hp, const int32_t* host_perms,
                   const dppo_learn_outputs* outputs, void* stream) {
  return learn_impl(h, rollout, params, adam_m, adam_v, hp, host_perms, false, outputs, stream);
}

int dppo_learn_targets_f32(dppo_handle* h, const dppo_rollout* rollout, float* params,
                           float* adam_m, float* adam_v, const dppo_hparams* hp,
                           const int32_t* host_targets, const dppo_learn_outputs* outputs,
                           void* stream) {
  return learn_impl(h, rollout, params, adam_m, adam_v, hp, host_targets, true, outputs, stream);
}

int dppo_global_minibatch_lists(dppo_handle* h, const int32_t* targets, int32_t* local,
                                int32_t* seg, void* stream) {
  if (!h || !targets || !local || !seg || !h->gmb) {
    set_error("dppo_global_minibatch_lists: needs a global_minibatches handle of world_size > 1 "
              "and device targets / local / seg buffers");
    return DPPO_EINVAL;
  }
  const dppo_dims& d = h->dims;
  if (h->Bg % d.num_minibatches != 0) {
    set_error("dppo_global_minibatch_lists: global batch %lld not divisible into %d minibatches",
              (long long)h->Bg, d.num_minibatches);
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  // the lists are built in the handle's own workspace (perms_dev as marks, perm_scratch,
  // sel_cnt), which a learn enqueued on another stream may still be reading
  DPPO_TRY(order_after_last(h, S(stream)));
  Timed tm(h, K_PERM, S(stream));
  if (perm_walk())
    return launch_shard_select_targets(targets, h->perms_dev, h->perm_scratch, h->perm_scratch_n,
                                       local, seg,
                                       h->sel_cnt, h->Bg, d.num_envs * d.world_size,
                                       d.num_envs * d.rank, d.num_envs, d.num_epochs,
                                       d.num_minibatches, S(stream));
  DPPO_TRY(launch_perm_resolve(targets, h->perms_dev, h->Bg, d.num_epochs, h->perm_scratch,
                               h->perm_scratch_n, S(stream)));
  return launch_shard_select(h->perms_dev, local, seg, h->sel_cnt, h->Bg,
                             d.num_envs * d.world_size, d.num_envs * d.rank, d.num_envs,
                             d.num_epochs, d.num_minibatches, S(stream));
}

int dppo_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                      int32_t* scratch, void* stream) {
  if (!targets || !perms || !scratch || n < 0 || n > 0x7FFFFFFF || count < 0) {
    set_error("invalid argument to dppo_perm_resolve");
    return DPPO_EINVAL;
  }
  return launch_perm_resolve(targets, perms, n, count, scratch, 3 * n * (int64_t)count,
                             S(stream));
}

int64_t dppo_perm_resolve_scratch(int64_t n, int32_t count) {
  if (n < 0 || n > 0x7FFFFFFF || count < 0) return -1;
  return perm_scratch_ints(n, count);
}

int dppo_perm_resolve_ex(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                         int32_t* scratch, int64_t scratch_ints, void* stream) {
  if (!targets || !perms || !scratch || n < 0 || n > 0x7FFFFFFF || count < 0 ||
      scratch_ints < 3 * n * (int64_t)count) {
    set_error("invalid argument to dppo_perm_resolve_ex (scratch_ints < 3 * count * n?)");
    return DPPO_EINVAL;
  }
  return launch_perm_resolve(targets, perms, n, count, scratch, scratch_ints, S(stream));
}

int dppo_perm_buffer(dppo_handle* h, int32_t slot, int32_t** out) {
  if (!h || !out || slot < 0 || slot >= kPermSlots) {
    set_error("invalid argument to dppo_perm_buffer");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  if (h->perm_copy_pending[slot]) {
    // Runs on the launching thread (engine._start_draft claims a slot before queueing its draft):
    // the slot's previous upload was enqueued two learns earlier and is normally long done, so
    // this is one hipEventQuery.  When it is not, it is polled with short sleeps rather than a
    // spinning hipEventSynchronize, which competes with the HIP runtime's submission threads
    // (measured on the draft thread: kernel enqueues 0.24 -> 0.55 ms per learn).
    hipError_t e;
    while ((e = hipEventQuery(h->perm_copy_done[slot])) == hipErrorNotReady)
      std::this_thread::sleep_for(std::chrono::microseconds(10));
    if (e != hipSuccess) {
      set_error("hipEventQuery: %s", hipGetErrorString(e));
      return DPPO_EHIP;
    }
    h->perm_copy_pending[slot] = false;
  }
  *out = h->perms_pinned[slot];
  return DPPO_OK;
}

int dppo_perm_external(dppo_handle* h, int32_t k, int32_t* ptr, int64_t bytes) {
  if (!h || k < 0 || k >= kExtSlots || (ptr && bytes <= 0)) {
    set_error("invalid argument to dppo_perm_external (slot 0..%d)", kExtSlots - 1);
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  if (h->ext_ptr[k]) {  // the previous registration: its upload must be done before unpinning
    if (h->ext_pending[k]) DPPO_HIP_CHECK(hipEventSynchronize(h->ext_done[k]));
    h->ext_pending[k] = false;
    DPPO_HIP_CHECK(hipHostUnregister(h->ext_ptr[k]));
    h->ext_ptr[k] = nullptr;
    h->ext_bytes[k] = 0;
  }
  if (!ptr) return DPPO_OK;
  if (!h->ext_done[k])
    DPPO_HIP_CHECK(hipEventCreateWithFlags(&h->ext_done[k], hipEventDisableTiming));
  const hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    set_error("hipHostRegister(%lld bytes) failed: %s", (long long)bytes, hipGetErrorString(e));
    return DPPO_EHIP;
  }
  h->ext_ptr[k] = ptr;
  h->ext_bytes[k] = bytes;
  return DPPO_OK;
}

int dppo_perm_external_done(dppo_handle* h, int32_t k, int32_t* done) {
  if (!h || !done || k < 0 || k >= kExtSlots) {
    set_error("invalid argument to dppo_perm_external_done");
    return DPPO_EINVAL;
  }
  *done = 1;
  if (!h->ext_pending[k]) return DPPO_OK;
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  const hipError_t e = hipEventQuery(h->ext_done[k]);
  if (e == hipErrorNotReady) {
    *done = 0;
    return DPPO_OK;
  }
  if (e != hipSuccess) {
    set_error("hipEventQuery: %s", hipGetErrorString(e));
    return DPPO_EHIP;
  }
  h->ext_pending[k] = false;
  return DPPO_OK;
}

int dppo_set_timing(dppo_handle* h, int32_t enable) {
  if (!h) {
    set_error("null handle");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  DPPO_HIP_CHECK(hipDeviceSynchronize());
  h->timing = enable != 0;
  h->recs.clear();
  h->pool_used = 0;
  return DPPO_OK;
}

int dppo_get_timing(dppo_handle* h, double* ms_sum, int64_t* counts) {
  if (!h || !ms_sum || !counts) {
    set_error("null argument to dppo_get_timing");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  for (int k = 0; k < DPPO_TIMING_CLASSES; ++k) {
    ms_sum[k] = 0.0;
    counts[k] = 0;
  }
  for (const auto& r : h->recs) {
    DPPO_HIP_CHECK(hipEventSynchronize(r.b));
    float ms = 0.f;
    DPPO_HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
    ms_sum[r.cls] += ms;
    counts[r.cls] += 1;
  }
  return DPPO_OK;
}

int dppo_get_trace(dppo_handle* h, float* host_out, int32_t rows) {
  if (!h || !host_out || rows < 0 || rows > h->trace_rows) {
    set_error("invalid argument to dppo_get_trace");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  DPPO_HIP_CHECK(hipStreamSynchronize(h->last_stream));
  DPPO_TRY(device_status(h));
  DPPO_HIP_CHECK(hipMemcpy(host_out, h->trace, (size_t)rows * DPPO_TRACE_FIELDS * sizeof(float),
                           hipMemcpyDeviceToHost));
  return DPPO_OK;
}

int dppo_comm_unique_id(char* out128) {
  if (!out128) {
    set_error("null argument");
    return DPPO_EINVAL;
  }
  ncclUniqueId id;
  DPPO_NCCL_CHECK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, 128);
  return DPPO_OK;
}

int dppo_comm_init(dppo_handle* h, int32_t nranks, int32_t rank, const char* id128) {
  if (!h || !id128 || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("invalid argument to dppo_comm_init");
    return DPPO_EINVAL;
  }
  if (h->comm || h->loop) {
    set_error("dppo_comm_init: the handle already has a communicator or loopback group");
    return DPPO_EINVAL;
  }
  if (h->gmb && nranks != h->dims.world_size) {
    set_error("dppo_comm_init: global_minibatches handle of world_size %d cannot join %d ranks",
              h->dims.world_size, nranks);
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  ncclUniqueId id;
  std::memcpy(&id, id128, 128);
  ncclComm_t c;
  DPPO_NCCL_CHECK(ncclCommInitRank(&c, nranks, id, rank));
  h->comm = c;
  h->nranks = nranks;
  h->rank = rank;
  return DPPO_OK;
}

// ---- peer exchange (peer.hip) ---------------------------------------------------------------
// Exchange buffers are never returned to the allocator: a destroyed handle's buffer goes to this
// process-wide pool and the next handle that needs one of the same size and memory type takes it
// (zeroed again).  Round 6: a coarse- or fine-grained exchange buffer created where
// freed uncached ones had been (twice the same virtual address range) lost the first store to one
// of its words for good -- a fault of address reuse below the memory model, which no fence or
// cache-policy bit cured; with the uncached buffers kept alive the same history stayed exact.
// Keeping every exchange buffer for the life of the process means no later allocation ever
// reuses one's address range.  (DPPO_PEER_NOPOOL=1 with DPPO_TEST_HOOKS=1: free as before, for
// tools/gpu/r06_coarse_diag.py.)
struct XPoolEntry {
  char* p;
  int64_t bytes;
  int mem;
  int device;
};
static std::mutex g_xpool_mu;
static std::vector<XPoolEntry> g_xpool;

static void xpool_put(dppo_handle* h) {
  if (!h->xbuf) return;
  if (test_hook("DPPO_PEER_NOPOOL")) {
    (void)hipFree(h->xbuf);
  } else {
    std::lock_guard<std::mutex> lk(g_xpool_mu);
    g_xpool.push_back({h->xbuf, h->xbytes, h->xmem, h->device});
  }
  h->xbuf = nullptr;
}

static char* xpool_take(int64_t bytes, int mem, int device) {
  std::lock_guard<std::mutex> lk(g_xpool_mu);
  for (size_t i = 0; i < g_xpool.size(); ++i) {
    const XPoolEntry e = g_xpool[i];
    if (e.bytes == bytes && e.mem == mem && e.device == device) {
      g_xpool.erase(g_xpool.begin() + (std::ptrdiff_t)i);
      return e.p;
    }
  }
  return nullptr;
}

static void peer_unmap(dppo_handle* h) {
  for (int r = 0; r < kMaxPeers; ++r) {
    if (h->xmapped[r]) (void)hipIpcCloseMemHandle(h->xpeer[r]);
    h->xmapped[r] = false;
    h->xpeer[r] = nullptr;
  }
  h->xworld = 0;
}

int dppo_peer_export(dppo_handle* h, unsigned char* out64) {
  if (!h || !out64) {
    set_error("invalid argument to dppo_peer_export");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  if (!h->xbuf) {
    const int64_t cap = h->layout.total + 8 > 64 ? h->layout.total + 8 : 64;
    if (cap > (int64_t)kPeerChunk * kPeerMaxSlices) {
      set_error("peer exchange: %lld parameters exceed the exchange's %d elements",
                (long long)cap, kPeerChunk * kPeerMaxSlices);
      return DPPO_EUNSUPPORTED;
    }
    // a whole 2 MiB allocation of its own (IPC maps allocations, not sub-ranges of a pool).
    // DPPO_PEER_MEM: uncached (hipDeviceMallocUncached, the default), fine
    // (hipDeviceMallocFinegrained) or coarse (hipMalloc).  Peers poll these words across xGMI
    // with system-scope loads; uncached memory is never held in any agent's L2, so a poll
    // always reads the owner's HBM and a publish is visible once its store retires -- coherent
    // across devices by construction, and measured no slower than coarse.
    const int64_t bytes = (peer_buffer_bytes(cap) + (2 << 20) - 1) / (2 << 20) * (2 << 20);
    const char* mem = std::getenv("DPPO_PEER_MEM");
    h->xmem = !mem ? 2 : (std::strcmp(mem, "fine") == 0 ? 1 : std::strcmp(mem, "coarse") == 0 ? 0 : 2);
    // One exchange-buffer memory type per process (round 6): a coarse- or
    // fine-grained exchange buffer created in a process that had created and freed two uncached
    // ones lost the first store to one of its words -- the word still read its initial zero 10 s
    // after the same lane had stored it, with or without a system-scope acquire (L1 / L2
    // invalidate) before every read, so no scope or cache-policy bit of the publish / poll can
    // restore it.  Every single-type history tested stayed exact; a second type is refused.
    static std::mutex xmem_mu;
    static int xmem_process = -1;
    {
      std::lock_guard<std::mutex> lk(xmem_mu);
      // (DPPO_PEER_MIX=1 with DPPO_TEST_HOOKS=1: allowed, for tools/gpu/r06_coarse_diag.py)
      if (xmem_process >= 0 && xmem_process != h->xmem && !test_hook("DPPO_PEER_MIX")) {
        static const char* kName[3] = {"coarse", "fine", "uncached"};
        set_error("dppo_peer_export: this process already created a%s %s exchange buffer; one of "
                  "type %s in the same process is refused (DPPO_PEER_MEM must not change within a "
                  "process: DESIGN.md section 6, round 6)",
                  xmem_process == 2 ? "n" : "", kName[xmem_process], kName[h->xmem]);
        return DPPO_EUNSUPPORTED;
      }
      xmem_process = h->xmem;
    }
    h->xbytes = bytes;
    if ((h->xbuf = xpool_take(bytes, h->xmem, h->device)) != nullptr) {
      // a pooled buffer of a destroyed handle (zeroed below)
    } else if (h->xmem == 0) {
      DPPO_TRY(dalloc(&h->xbuf, bytes));
    } else {
      const hipError_t e = hipExtMallocWithFlags((void**)&h->xbuf, (size_t)bytes,
                                                 h->xmem == 1 ? hipDeviceMallocFinegrained
                                                              : hipDeviceMallocUncached);
      if (e != hipSuccess) {
        h->xbuf = nullptr;
        set_error("hipExtMallocWithFlags(%lld bytes, %s) failed: %s", (long long)bytes,
                  h->xmem == 1 ? "fine-grained" : "uncached", hipGetErrorString(e));
        return DPPO_ENOMEM;
      }
    }
    DPPO_HIP_CHECK(hipMemset(h->xbuf, 0, (size_t)bytes));
    if (const char* dbg = std::getenv("DPPO_PEER_DEBUG"))
      if (dbg[0] == '1')
        std::fprintf(stderr, "dppo peer: exchange buffer %p, %lld bytes, memory type %d\n",
                     (void*)h->xbuf, (long long)bytes, h->xmem);
    // DPPO_PEER_XSEQ0 (test hook, dppo_peer_open): counting on from s0, the slice flags start as
    // if exchange s0 had just completed -- the (wrap-safe) flag comparison needs flags within
    // 2^31 of the sequence, as they always are once exchanges have run
    if (const char* x0 = test_hook("DPPO_PEER_XSEQ0")) {
      const unsigned s0 = (unsigned)std::strtoul(x0, nullptr, 0);
      for (int k = 0; k < kPeerMaxSlices; ++k)
        DPPO_HIP_CHECK(hipMemcpy(h->xbuf + 4 * cap * 8 + 64 * (int64_t)k, &s0, sizeof(s0),
                                 hipMemcpyHostToDevice));
    }
    DPPO_HIP_CHECK(hipDeviceSynchronize());
    h->xcap = cap;
  }
  hipIpcMemHandle_t hd;
  static_assert(sizeof(hd) == 64, "hipIpcMemHandle_t size");
  if (test_hook("DPPO_PEER_NOIPC")) {  // (diagnosis, 1-rank exchanges only: no IPC export)
    std::memset(out64, 0, 64);
    return DPPO_OK;
  }
  DPPO_HIP_CHECK(hipIpcGetMemHandle(&hd, h->xbuf));
  std::memcpy(out64, &hd, 64);
  return DPPO_OK;
}

int dppo_peer_open(dppo_handle* h, int32_t nranks, int32_t rank, const unsigned char* handles,
                   int32_t flags) {
  if (!h || !handles || nranks < 1 || nranks > kMaxPeers || rank < 0 || rank >= nranks) {
    set_error("invalid argument to dppo_peer_open (1..%d ranks)", kMaxPeers);
    return DPPO_EINVAL;
  }
  if (!h->xbuf || h->xworld > 0 || h->loop) {
    set_error("dppo_peer_open: needs dppo_peer_export first, no open exchange, no loopback group");
    return DPPO_EINVAL;
  }
  if (h->comm && (nranks != h->nranks || rank != h->rank)) {
    set_error("dppo_peer_open: rank %d of %d disagrees with the communicator's %d of %d", rank,
              nranks, h->rank, h->nranks);
    return DPPO_EINVAL;
  }
  if (h->gmb && nranks != h->dims.world_size) {
    set_error("dppo_peer_open: global_minibatches handle of world_size %d cannot join %d ranks",
              h->dims.world_size, nranks);
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  for (int r = 0; r < nranks; ++r) {
    if (r == rank) {
      h->xpeer[r] = h->xbuf;
      continue;
    }
    hipIpcMemHandle_t hd;
    std::memcpy(&hd, handles + 64 * r, 64);
    void* p = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&p, hd, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      peer_unmap(h);
      set_error("dppo_peer_open: mapping rank %d's exchange buffer failed: %s", r,
                hipGetErrorString(e));
      return DPPO_ECOMM;
    }
    h->xpeer[r] = (char*)p;
    h->xmapped[r] = true;
  }
  const char* t = std::getenv("DPPO_PEER_TIMEOUT_S");
  const double sec = t ? std::atof(t) : 60.0;
  h->xticks = (unsigned long long)((sec > 0.0 ? sec : 60.0) * 1e8);
  // The fused form needs every rank's reduce_adam grid resident at once: true with one GPU per
  // rank, not when ranks share a device (their grids would wait on each other for CUs).
  const char* fz = std::getenv("DPPO_PEER_FUSED");
  h->xfused = !(flags & DPPO_PEER_SHARED_DEVICE) && !(fz && fz[0] == '0');
  // DPPO_PEER_XSEQ0 (tests): the exchange number to count on from, e.g. just below the 32-bit
  // wrap; every rank must set the same value
  const char* x0 = test_hook("DPPO_PEER_XSEQ0");
  if (x0) h->xseq = (unsigned)std::strtoul(x0, nullptr, 0);
  h->xworld = nranks;
  h->nranks = nranks;
  h->rank = rank;
  return DPPO_OK;
}

int dppo_peer_close(dppo_handle* h) {
  if (!h) {
    set_error("invalid argument to dppo_peer_close");
    return DPPO_EINVAL;
  }
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  DPPO_HIP_CHECK(hipDeviceSynchronize());
  peer_unmap(h);
  // a failed exchange (e.g. the self-test) leaves nothing in flight after the synchronisation:
  // the handle is usable again on its other transport
  if (h->err_host && (__atomic_load_n(h->err_host, __ATOMIC_ACQUIRE) & 0xffu) == kErrPeerTimeout)
    __atomic_store_n(h->err_host, 0u, __ATOMIC_RELEASE);
  if (!h->comm) {
    h->nranks = h->dims.world_size;
    h->rank = h->dims.rank;
  }
  return DPPO_OK;
}

int dppo_peer_info(dppo_handle* h, int64_t* out4) {
  if (!h || !out4) {
    set_error("invalid argument to dppo_peer_info");
    return DPPO_EINVAL;
  }
  out4[0] = h->xworld;
  out4[1] = h->xworld > 0 && h->xfused && h->radam_ok ? 1 : 0;
  out4[2] = h->xbuf ? h->xmem : -1;
  out4[3] = (int64_t)h->xseq;
  return DPPO_OK;
}

int dppo_peer_allreduce(dppo_handle* h, void* buf, int64_t n, int32_t f64, void* stream) {
  if (!h || !buf || n < 1) {
    set_error("invalid argument to dppo_peer_allreduce");
    return DPPO_EINVAL;
  }
  if (h->xworld < 1) {
    set_error("dppo_peer_allreduce: no open peer exchange (dppo_peer_open)");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  return peer_allreduce(h, buf, (size_t)n, f64 != 0, S(stream));
}

int dppo_peer_selftest(dppo_handle* h, void* stream) {
  if (!h || h->xworld < 1) {
    set_error("dppo_peer_selftest: no open peer exchange (dppo_peer_open)");
    return DPPO_EINVAL;
  }
  DPPO_TRY(device_status(h));
  DPPO_HIP_CHECK(hipSetDevice(h->device));
  hipStream_t s = S(stream);
  const int W = h->xworld;
  const int tri = W * (W + 1) / 2;
  const int64_t n = h->layout.total + 8;
  // Exchange k (k = 0..3, both buffer parities twice, so every exchange after the first two
  // overwrites non-zero words of an earlier one): rank r contributes (r + 1) (i % 7 + 1) + 1000 k
  // in f32 -- exact sums tri (i % 7 + 1) + 1000 W k -- and exchange 0 also (r + 1) {0.25, -0.5}
  // in f64.  Then, where the learn runs the gradient exchange inside reduce_adam_kernel (one GPU
  // per rank), two launches of that kernel on a one-slab scratch gradient (r + 1) (i % 5 + 1) +
  // 100 k, both parities: its tagged-word sum must come out exact as well.
  std::vector<float> hf((size_t)n);
  double hd[2];
  float* df = nullptr;
  double* dd = nullptr;
  float *slab = nullptr, *pm = nullptr, *grad = nullptr;
  const bool fused = h->xfused && h->radam_ok && h->ra_tags;
  auto run = [&]() -> int {
    DPPO_TRY(dalloc(&df, n));
    DPPO_TRY(dalloc(&dd, 2));
    if (fused) {
      DPPO_TRY(dalloc(&slab, h->slab_stride));
      DPPO_TRY(dalloc(&pm, 3 * h->layout.total));
      DPPO_TRY(dalloc(&grad, n));
    }
    // DPPO_PEER_SELFTEST_SKEW=r (tests): rank r contributes one wrong element to exchange 0, as
    // a rank reading stale or incoherent peer memory would see it
    const char* skew = test_hook("DPPO_PEER_SELFTEST_SKEW");
    const int skew_rank = skew ? std::atoi(skew) : -1;
    for (int k = 0; k < 4; ++k) {
      for (int64_t i = 0; i < n; ++i)
        hf[i] = (float)((h->rank + 1) * (int)(i % 7 + 1) + 1000 * k);
      if (k == 0 && skew_rank == h->rank) hf[3] += 1.0f;
      DPPO_HIP_CHECK(hipMemcpyAsync(df, hf.data(), n * 4, hipMemcpyHostToDevice, s));
      DPPO_TRY(peer_allreduce(h, df, (size_t)n, false, s));
      if (k == 0) {
        hd[0] = (h->rank + 1) * 0.25;
        hd[1] = -(h->rank + 1) * 0.5;
        DPPO_HIP_CHECK(hipMemcpyAsync(dd, hd, 16, hipMemcpyHostToDevice, s));
        DPPO_TRY(peer_allreduce(h, dd, 2, true, s));
        DPPO_HIP_CHECK(hipMemcpyAsync(hd, dd, 16, hipMemcpyDeviceToHost, s));
      }
      DPPO_HIP_CHECK(hipMemcpyAsync(hf.data(), df, n * 4, hipMemcpyDeviceToHost, s));
      DPPO_HIP_CHECK(hipStreamSynchronize(s));
      DPPO_TRY(device_status(h));
      for (int64_t i = 0; i < n; ++i) {
        const float want = (float)(tri * (int)(i % 7 + 1) + 1000 * W * k);
        if (hf[i] != want) {
          set_error("peer exchange self-test: exchange %d element %lld is %g, expected %g", k,
                    (long long)i, (double)hf[i], (double)want);
          return DPPO_ECOMM;
        }
      }
      if (k == 0 && (hd[0] != tri * 0.25 || hd[1] != -tri * 0.5)) {
        set_error("peer exchange self-test: f64 sums %g %g, expected %g %g", hd[0], hd[1],
                  tri * 0.25, -tri * 0.5);
        return DPPO_ECOMM;
      }
    }
    if (!fused) return DPPO_OK;
    const int64_t P = h->layout.total;
    DPPO_HIP_CHECK(hipMemsetAsync(pm, 0, 3 * P * sizeof(float), s));
    for (int k = 0; k < 2; ++k) {
      for (int64_t i = 0; i < n; ++i)
        hf[i] = (float)((h->rank + 1) * (int)(i % 5 + 1) + 100 * k);
      DPPO_HIP_CHECK(hipMemcpyAsync(slab, hf.data(), n * 4, hipMemcpyHostToDevice, s));
      PeerArgs pa{};
      for (int r = 0; r < W; ++r) pa.bufs[r] = h->xpeer[r];
      pa.data_bytes = h->xcap * 8;
      pa.world = W;
      pa.rank = h->rank;
      pa.seq = next_xseq(h);
      pa.err = h->err_dev;
      pa.timeout_ticks = h->xticks;
          pa.acq = peer_acq();
      DPPO_TRY(launch_reduce_adam(slab, 1, h->slab_stride, P, grad, h->ra_tags, 0, 0, 0.f, 0,
                                  next_radam_epoch(h), pm, pm + P, pm + 2 * P, 0.5f, -1e-3f, 1.f,
                                  0.9f, 0.999f, 1e-5f, nullptr, 1.f, 1.f, 0.f, h->err_dev,
                                  h->xticks, s, &pa));
      DPPO_HIP_CHECK(hipMemcpyAsync(hf.data(), grad, n * 4, hipMemcpyDeviceToHost, s));
      DPPO_HIP_CHECK(hipStreamSynchronize(s));
      DPPO_TRY(device_status(h));
      for (int64_t i = 0; i < n; ++i) {
        const float want = (float)(tri * (int)(i % 5 + 1) + 100 * W * k);
        if (hf[i] != want) {
          set_error("peer exchange self-test: fused exchange %d element %lld is %g, expected %g",
                    k, (long long)i, (double)hf[i], (double)want);
          return DPPO_ECOMM;
        }
      }
    }
    return DPPO_OK;
  };
  // a peer that cannot see our buffer fails the test in seconds, not after the learn's bound
  const unsigned long long ticks = h->xticks;
  if (h->xticks > 1000000000ull) h->xticks = 1000000000ull;
  const int rc = run();
  h->xticks = ticks;
  (void)hipStreamSynchronize(s);
  for (void* p : {(void*)df, (void*)dd, (void*)slab, (void*)pm, (void*)grad})
    if (p) (void)hipFree(p);
  return rc;
}

int dppo_loopback_group(dppo_handle** hs, int32_t n) {
  if (!hs || n < 2 || n > kMaxLoopRanks) {
    set_error("dppo_loopback_group: need 2..%d handles", kMaxLoopRanks);
    return DPPO_EINVAL;
  }
  for (int r = 0; r < n; ++r) {
    dppo_handle* h = hs[r];
    if (!h || h->device != hs[0]->device || h->nranks != n || h->rank != r || h->comm ||
        h->loop || h->layout.total != hs[0]->layout.total) {
      set_error("dppo_loopback_group: handle %d must be rank %d of world_size %d on device %d, "
                "same parameter layout, no communicator or group yet", r, r, n, hs[0]->device);
      return DPPO_EINVAL;
    }
  }
  auto g = std::make_shared<LoopGroup>();
  g->n = n;
  for (int r = 0; r < n; ++r) {
    dppo_handle* h = hs[r];
    DPPO_HIP_CHECK(hipSetDevice(h->device));
    h->loop_bytes = std::max<size_t>((size_t)h->slab_stride * sizeof(float), 4 * sizeof(double));
    DPPO_HIP_CHECK(hipMalloc(&h->loop_out, h->loop_bytes));
    DPPO_HIP_CHECK(hipEventCreateWithFlags(&h->loop_ready, hipEventDisableTiming));
    DPPO_HIP_CHECK(hipEventCreateWithFlags(&h->loop_done, hipEventDisableTiming));
    g->members[r] = h;
  }
  for (int r = 0; r < n; ++r) hs[r]->loop = g;
  return DPPO_OK;
}

}  // extern "C"
