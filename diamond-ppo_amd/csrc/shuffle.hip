// Fisher-Yates resolution on the device: minibatch permutations from their swap targets.
//
// np.random.permutation(n) (reference diamond/ppo.py:254; numpy legacy RandomState) is the
// sequential shuffle   a = arange(n); for i = n-1 .. 1: swap(a[i], a[j_i])   with j_i <= i drawn
// from MT19937 by rejection (perm.cpp draws the j_i on the host, bit-exactly).  The swaps are a
// dependent chain on the host (~1.4 ms per 4 x 524288 on a 5 GHz core); here they are resolved
// in parallel with the closed form of the shuffle:
//
//   position i is final after step i, and before step i position p < i holds the value last
//   written into it, i.e. by the latest step i'' > i with j_i'' = p (or p itself if none).
//   With  succ(i) = min{ i'' > i : j_i'' = j_i }   and   M(q) = min{ i'' > q : j_i'' = q }:
//     W(q)   = value at position q just before step q = root(q)  (follow M until it is absent)
//     out[i] = succ(i) exists ? W(succ(i)) : j_i          (i >= 1)
//     out[0] = W(0)
//
// Three grid-stride passes over count*n elements (HBM/L2-latency bound, no MFMA):
//   build : per-target linked lists   head[c][p] <- i   (atomicExch; list order irrelevant)
//   links : M(x) from bucket x, succ(x) from bucket j_x   (bucket sizes ~ ln(n/p), tiny)
//   solve : out = W(succ) / j / W(0)   (chains strictly increase, length ~ ln n)
// Every value is a min over a set, so the result is deterministic despite the atomics.
#include "common.h"

namespace dppo {
namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void fy_build_kernel(const int32_t* __restrict__ tgt,
                                                         int32_t* __restrict__ head,
                                                         int32_t* __restrict__ nxt, int64_t n,
                                                         int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int32_t i = (int32_t)(g - c * n);
    const int32_t p = tgt[g];
    int32_t prev = -1;
    // i = 0 takes no step; a target outside [0, i] (never produced by the host draw) is ignored
    // rather than allowed to index out of range
    if (i > 0 && (uint32_t)p <= (uint32_t)i) prev = atomicExch(&head[c * n + p], i);
    nxt[g] = prev;
  }
}

__device__ __forceinline__ int32_t min_above(const int32_t* __restrict__ head,
                                             const int32_t* __restrict__ nxt, int64_t base,
                                             int32_t bucket, int32_t x) {
  int32_t best = 0x7FFFFFFF;
  for (int32_t it = head[base + bucket]; it >= 0; it = nxt[base + it])
    best = (it > x && it < best) ? it : best;
  return best == 0x7FFFFFFF ? -1 : best;
}

__global__ __launch_bounds__(kBlock) void fy_links_kernel(const int32_t* __restrict__ tgt,
                                                         const int32_t* __restrict__ head,
                                                         const int32_t* __restrict__ nxt,
                                                         int32_t* __restrict__ mq,
                                                         int32_t* __restrict__ succ, int64_t n,
                                                         int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int64_t base = c * n;
    const int32_t x = (int32_t)(g - base);
    mq[g] = min_above(head, nxt, base, x, x);
    int32_t s = -1;
    const int32_t p = tgt[g];
    if (x > 0 && (uint32_t)p <= (uint32_t)x) s = min_above(head, nxt, base, p, x);
    succ[g] = s;
  }
}

__device__ __forceinline__ int32_t root(const int32_t* __restrict__ mq, int64_t base, int32_t q) {
  for (int32_t m = mq[base + q]; m >= 0; m = mq[base + q]) q = m;
  return q;
}

// The value walk (the inverse form of the closed form above): value v starts at position q = v
// with every step i >= n still to come.  The first step that touches position q is the LARGEST
// step i in (q, bound) with j_i = q -- it moves v up to position i, which no later (smaller)
// step can touch: final -- and otherwise step q itself, which moves v down to j_q (or leaves it:
// j_q = q, final); from there only steps below the old q remain.  Positions strictly decrease, so
// the walk ends; on random targets it takes ~2 hops of ~2 bucket entries each (NumPy
// restatement: tests/test_native_cpu.py value_walk_positions).  A rank that needs the positions of only some values
// (global minibatches: its own env shard) walks only those.
__device__ __forceinline__ int32_t walk_pos(const int32_t* __restrict__ tgt,
                                            const int32_t* __restrict__ head,
                                            const int32_t* __restrict__ nxt, int64_t base,
                                            int32_t n, int32_t v) {
  int32_t q = v, bound = n;
  for (;;) {
    int32_t best = -1;
    for (int32_t it = head[base + q]; it >= 0; it = nxt[base + it])
      best = (it > q && it < bound && it > best) ? it : best;
    if (best >= 0 || q == 0) return best >= 0 ? best : 0;
    const int32_t jq = tgt[base + q];
    if ((uint32_t)jq >= (uint32_t)q) return q;  // j_q == q (or an invalid target: stays)
    bound = q;
    q = jq;
  }
}

// perms[c][pos(v)] = v for every value: the whole permutation (one GPU)
__global__ __launch_bounds__(kBlock) void fy_walk_scatter_kernel(const int32_t* __restrict__ tgt,
                                                                const int32_t* __restrict__ head,
                                                                const int32_t* __restrict__ nxt,
                                                                int32_t* __restrict__ perms,
                                                                int64_t n, int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int32_t v = (int32_t)(g - c * n);
    perms[c * n + walk_pos(tgt, head, nxt, c * n, (int32_t)n, v)] = v;
  }
}

// marks[c][pos(v)] = l for this rank's values only: local sample l = t * nl + e of the shard
// [env0, env0 + nl) is global sample v = t * ng + env0 + e (marks pre-filled with -1)
__global__ __launch_bounds__(kBlock) void fy_walk_mark_kernel(const int32_t* __restrict__ tgt,
                                                             const int32_t* __restrict__ head,
                                                             const int32_t* __restrict__ nxt,
                                                             int32_t* __restrict__ marks,
                                                             int64_t n, int64_t b_local,
                                                             int32_t E, int32_t ng, int32_t env0,
                                                             int32_t nl) {
  const int64_t total = b_local * E;
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / b_local;
    const int32_t l = (int32_t)(g - c * b_local);
    const int32_t t = l / nl;
    const int32_t v = t * ng + env0 + (l - t * nl);
    marks[c * n + walk_pos(tgt, head, nxt, c * n, (int32_t)n, v)] = l;
  }
}

// out aliases succ (each thread reads its own succ before overwriting it)
__global__ __launch_bounds__(kBlock) void fy_solve_kernel(const int32_t* __restrict__ tgt,
                                                         const int32_t* __restrict__ mq,
                                                         int32_t* out, int64_t n, int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int64_t base = c * n;
    const int32_t x = (int32_t)(g - base);
    int32_t v;
    if (x == 0) {
      v = root(mq, base, 0);
    } else {
      const int32_t s = out[g];
      v = s >= 0 ? root(mq, base, s) : tgt[g];
    }
    out[g] = v;
  }
}

// ---- Global-minibatch data parallelism (dims.global_minibatches).
// Every rank holds the SAME E permutations of the global batch (reference ppo.py:252-255 over
// Bg = T*Ng samples, global flat index i = t*Ng + n).  Rank r keeps, in permutation order, the
// members of each global minibatch whose env n is in its shard [env0, env0 + Nl), as local flat
// indices t*Nl + (n - env0).  Per epoch the kept indices are a permutation of the rank's B = T*Nl
// samples grouped by global minibatch; seg[e][j] is where minibatch j starts, seg[e][M] = B.
// Two coalesced passes over the E*Bg ints, chunk-parallel over the whole chip:
//   count : matches per 16,384-element chunk
//   write : chunk start = sum of the epoch's earlier chunk counts; an ordered (ballot / mbcnt)
//           compaction per 256-element slice; the thread holding position j*mbg records seg[e][j]
constexpr int kSelPer = 64;                    // slices per chunk
constexpr int kSelChunk = kBlock * kSelPer;    // 16,384 elements

__device__ __forceinline__ bool in_shard(int32_t i, int32_t ng, int32_t env0, int32_t nl) {
  const int32_t t = i / ng;
  return (uint32_t)(i - t * ng - env0) < (uint32_t)nl;
}

// MARK: the source is a marks array (>= 0: this rank's local sample at that position) instead of
// the global permutation
template <bool MARK>
__device__ __forceinline__ bool sel_keep(int32_t x, int32_t ng, int32_t env0, int32_t nl) {
  return MARK ? x >= 0 : in_shard(x, ng, env0, nl);
}

template <bool MARK>
__global__ __launch_bounds__(kBlock) void shard_count_kernel(const int32_t* __restrict__ gperm,
                                                            int32_t* __restrict__ cnt, int64_t bg,
                                                            int32_t ng, int32_t env0, int32_t nl) {
  __shared__ int32_t wsum[kBlock / 64];
  const int64_t e = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * kSelChunk;
  const int32_t* src = gperm + e * bg;
  int32_t k = 0;
  for (int s = 0; s < kSelPer; ++s) {
    const int64_t p = c0 + (int64_t)s * kBlock + threadIdx.x;
    if (p < bg && sel_keep<MARK>(src[p], ng, env0, nl)) ++k;
  }
  for (int off = 32; off >= 1; off >>= 1) k += __shfl_xor(k, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = k;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += wsum[w];
    cnt[e * gridDim.x + blockIdx.x] = t;
  }
}

template <bool MARK>
__global__ __launch_bounds__(kBlock) void shard_write_kernel(
    const int32_t* __restrict__ gperm, const int32_t* __restrict__ cnt,
    int32_t* __restrict__ local, int32_t* __restrict__ seg, int64_t bg, int32_t ng, int32_t env0,
    int32_t nl, int32_t M) {
  __shared__ int32_t red[kBlock / 64];
  __shared__ int32_t wtot[2][kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t e = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * kSelChunk;
  const int32_t* src = gperm + e * bg;
  const int64_t B = (int64_t)(bg / ng) * nl;
  const int64_t mbg = bg / M;
  // start of this chunk in the epoch's local list
  int32_t before = 0;
  for (int c = threadIdx.x; c < (int)blockIdx.x; c += kBlock) before += cnt[e * gridDim.x + c];
  for (int off = 32; off >= 1; off >>= 1) before += __shfl_xor(before, off);
  if (lane == 0) red[wave] = before;
  __syncthreads();
  int32_t base = 0;
  for (int w = 0; w < kBlock / 64; ++w) base += red[w];
  int32_t* out = local + e * B;
  for (int s = 0; s < kSelPer; ++s) {
    const int64_t p = c0 + (int64_t)s * kBlock + threadIdx.x;
    int32_t i = 0;
    bool keep = false;
    if (p < bg) {
      i = src[p];
      keep = sel_keep<MARK>(i, ng, env0, nl);
    }
    const unsigned long long mask = __ballot(keep);
    const int32_t pre = (int32_t)__builtin_amdgcn_mbcnt_hi(
        (unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    if (lane == 0) wtot[s & 1][wave] = (int32_t)__popcll(mask);
    __syncthreads();
    int32_t wpre = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      const int32_t x = wtot[s & 1][w];
      wpre += w < wave ? x : 0;
      tot += x;
    }
    const int32_t pos = base + wpre + pre;  // kept samples before position p in this epoch
    if (keep) {
      if (MARK) {
        out[pos] = i;
      } else {
        const int32_t t = i / ng;
        out[pos] = t * nl + (i - t * ng - env0);
      }
    }
    if (p < bg && p % mbg == 0) seg[e * (M + 1) + p / mbg] = pos;
    base += tot;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) seg[e * (M + 1) + M] = (int32_t)B;
}

int fy_grid(int64_t total) {
  int64_t b = (total + kBlock - 1) / kBlock;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

}  // namespace

// DPPO_PERM_WALK: 1 = the value walk, 0 = the links + solve passes.  One GPU (the whole
// permutation) defaults to the passes: C5's 4 x 8.4 M took 4.06-4.10 ms per learn with them
// against 4.75-4.93 with the walk (round 5, 2 A/B reps) -- the walk's hops are dependent loads.
// Global minibatches default to the walk: a rank walks only its 1/world of the values.
bool perm_walk_env(bool dflt) {
  const char* e = std::getenv("DPPO_PERM_WALK");
  return e ? e[0] != '0' : dflt;
}
bool perm_walk() { return perm_walk_env(true); }

int launch_perm_resolve_one(const int32_t* targets, int32_t* perms, int64_t n, int32_t* scratch,
                            hipStream_t s) {
  int32_t* head = scratch;
  int32_t* nxt = scratch + n;
  int32_t* mq = scratch + 2 * n;
  DPPO_HIP_CHECK(hipMemsetAsync(head, 0xFF, (size_t)n * sizeof(int32_t), s));
  const int G = fy_grid(n);
  DPPO_LAUNCH(fy_build_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, n, n);
  DPPO_LAUNCH_CHECK();
  if (perm_walk_env(false)) {
    DPPO_LAUNCH(fy_walk_scatter_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, perms, n,
                n);
    DPPO_LAUNCH_CHECK();
    return DPPO_OK;
  }
  DPPO_LAUNCH(fy_links_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, mq, perms, n, n);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(fy_solve_kernel, dim3(G), dim3(kBlock), 0, s, targets, mq, perms, n, n);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int launch_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                        int32_t* scratch, hipStream_t s) {
  const int64_t total = n * (int64_t)count;
  if (total == 0) return DPPO_OK;
  // DPPO_PERM_EPOCHWISE=1 (A/B): one epoch at a time, so the random accesses of the three passes
  // (heads, links, chains: ~134 MB per 8.4 M-entry epoch) stay within the 256 MB Infinity Cache
  // instead of spanning all epochs' 536 MB at C5
  static const bool epochwise = [] {
    const char* e = std::getenv("DPPO_PERM_EPOCHWISE");
    return e && e[0] == '1';
  }();
  if (epochwise && count > 1) {
    for (int32_t c = 0; c < count; ++c) {
      const int rc = launch_perm_resolve_one(targets + c * n, perms + c * n, n, scratch, s);
      if (rc != DPPO_OK) return rc;
    }
    return DPPO_OK;
  }
  int32_t* head = scratch;
  int32_t* nxt = scratch + total;
  int32_t* mq = scratch + 2 * total;
  DPPO_HIP_CHECK(hipMemsetAsync(head, 0xFF, (size_t)total * sizeof(int32_t), s));
  const int G = fy_grid(total);
  DPPO_LAUNCH(fy_build_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, n, total);
  DPPO_LAUNCH_CHECK();
  if (perm_walk_env(false)) {
    DPPO_LAUNCH(fy_walk_scatter_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, perms, n,
                total);
    DPPO_LAUNCH_CHECK();
    return DPPO_OK;
  }
  DPPO_LAUNCH(fy_links_kernel, dim3(G), dim3(kBlock), 0, s, targets, head, nxt, mq, perms, n, total);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(fy_solve_kernel, dim3(G), dim3(kBlock), 0, s, targets, mq, perms, n, total);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

int shard_select_chunks(int64_t bg) { return (int)((bg + kSelChunk - 1) / kSelChunk); }

int launch_shard_select(const int32_t* gperm, int32_t* local, int32_t* seg, int32_t* cnt,
                        int64_t bg, int32_t ng, int32_t env0, int32_t nl, int32_t E, int32_t M,
                        hipStream_t s) {
  if (bg <= 0 || E <= 0) return DPPO_OK;
  const dim3 grid((unsigned)shard_select_chunks(bg), (unsigned)E);
  DPPO_LAUNCH(shard_count_kernel<false>, grid, dim3(kBlock), 0, s, gperm, cnt, bg, ng, env0, nl);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(shard_write_kernel<false>, grid, dim3(kBlock), 0, s, gperm, cnt, local, seg, bg, ng,
              env0, nl, M);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

// Global minibatches from swap targets without resolving the whole permutation: this rank's
// members of every global minibatch, in permutation order -- the same lists launch_shard_select
// makes from the resolved permutation.  scratch: 2 * E * bg ints (bucket heads and links); marks:
// E * bg ints.
int launch_shard_select_targets(const int32_t* targets, int32_t* marks, int32_t* scratch,
                                int32_t* local, int32_t* seg, int32_t* cnt, int64_t bg, int32_t ng,
                                int32_t env0, int32_t nl, int32_t E, int32_t M, hipStream_t s) {
  if (bg <= 0 || E <= 0) return DPPO_OK;
  const int64_t total = bg * E;
  int32_t* head = scratch;
  int32_t* nxt = scratch + total;
  DPPO_HIP_CHECK(hipMemsetAsync(head, 0xFF, (size_t)total * sizeof(int32_t), s));
  DPPO_HIP_CHECK(hipMemsetAsync(marks, 0xFF, (size_t)total * sizeof(int32_t), s));
  DPPO_LAUNCH(fy_build_kernel, dim3(fy_grid(total)), dim3(kBlock), 0, s, targets, head, nxt, bg,
              total);
  DPPO_LAUNCH_CHECK();
  const int64_t b_local = (bg / ng) * nl;
  DPPO_LAUNCH(fy_walk_mark_kernel, dim3(fy_grid(b_local * E)), dim3(kBlock), 0, s, targets, head,
              nxt, marks, bg, b_local, E, ng, env0, nl);
  DPPO_LAUNCH_CHECK();
  const dim3 grid((unsigned)shard_select_chunks(bg), (unsigned)E);
  DPPO_LAUNCH(shard_count_kernel<true>, grid, dim3(kBlock), 0, s, marks, cnt, bg, ng, env0, nl);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(shard_write_kernel<true>, grid, dim3(kBlock), 0, s, marks, cnt, local, seg, bg, ng,
              env0, nl, M);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
