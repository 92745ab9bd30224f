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
// The buckets (the steps with j_i = q, ~ln(n/q) of them) come from a partitioned counting sort
// (csr_* below, the default): histograms, prefixes and a scatter by target partition, then one
// workgroup per partition sorting its steps into contiguous buckets in LDS, M(q) per position,
// and the solve bucket by bucket.  Where that does not fit (tiny or very large n), three
// grid-stride passes over count*n elements instead (HBM/L2-latency bound, no MFMA):
//   build : per-target linked lists   head[c][p] <- i   (atomicExch; list order irrelevant)
//   links : M(x) from bucket x, succ(x) from bucket j_x   (bucket sizes ~ ln(n/p), tiny)
//   solve : out = W(succ) / j / W(0)   (chains strictly increase, length ~ ln n)
// Every value is a min over a set, so the result is deterministic despite the atomics.
#include "common.h"

#include <cstdint>

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

// ---- Buckets by a partitioned counting sort (the default where it fits; DPPO_PERM_CSR=0: the
// linked lists above).  The linked-list build is one random device-scope atomicExch per step
// (33.5 M at C5: 1.3 ms) and every later bucket read chases `nxt` pointers across 134 MB (the
// links pass fetched 15.9 GB for 4 x 8.4 M steps: 2.2 ms).  Here the positions are cut into
// partitions of P = 2^logp (<= 4096 per epoch) and the steps are sorted by target in two levels,
// every count in LDS:
//   count   : per chunk of 32,768 steps, an LDS histogram of the steps' target partitions
//   colscan : per partition, the exclusive prefix of its counts over the chunks
//   basescan: the partitions' starts in the sorted order (one block)
//   scatter : every valid step i (0 < i, j_i <= i) to its partition's range: (i, j_i mod P)
//   fill    : per partition, an LDS counting sort by position -> the partition's buckets
//             contiguous (bucket q = the steps with j_i = q, in no particular order)
//   index   : per position, M(q) = min{i > q in bucket q} and, for every step i of the bucket,
//             succ(i) = its next larger step (the resolution; fused with fill, in LDS, where the
//             scratch allows), or the bucket's start (the value walk)
//   solve   : fy_solve_kernel (out[i] = W(succ(i)) or j_i), or the value walk over the buckets
// Every bucket value is a min / max over a set, so the results are the same bits as the
// linked-list passes'.  Scratch layouts: csr_plan.
constexpr int kCsrChunk = 32768;    // steps per count / scatter workgroup
constexpr int kCsrMaxParts = 4096;  // partitions per epoch (count / scatter LDS: 16 KB)
constexpr int kCsrMinLogP = 11, kCsrMaxLogP = 12;  // P = 2048 .. 4096 (fill: 2P ints of LDS)

__global__ __launch_bounds__(kBlock) void csr_count_kernel(const int32_t* __restrict__ tgt,
                                                          int32_t* __restrict__ hist, int64_t n,
                                                          int64_t bpe, int logp, int nparts) {
  extern __shared__ int32_t h[];  // [nparts]
  const int64_t c = blockIdx.x / bpe, k = blockIdx.x - c * bpe;
  for (int x = threadIdx.x; x < nparts; x += kBlock) h[x] = 0;
  __syncthreads();
  const int32_t* t = tgt + c * n;
  const int64_t i0 = k * kCsrChunk, i1 = i0 + kCsrChunk < n ? i0 + kCsrChunk : n;
  for (int64_t ib = i0; ib < i1; ib += 8 * kBlock) {
    int32_t p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = ib + u * kBlock + threadIdx.x;
      p[u] = i < i1 ? t[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = ib + u * kBlock + threadIdx.x;
      if (i < i1 && i > 0 && (uint32_t)p[u] <= (uint32_t)i) atomicAdd(&h[p[u] >> logp], 1);
    }
  }
  __syncthreads();
  int32_t* row = hist + (int64_t)blockIdx.x * nparts;
  for (int x = threadIdx.x; x < nparts; x += kBlock) row[x] = h[x];
}

// thread g = partition (c, x): the exclusive prefix of hist[c][k][x] over the chunks k, in place;
// its total to tot[g]
__global__ __launch_bounds__(kBlock) void csr_colscan_kernel(int32_t* __restrict__ hist,
                                                            int32_t* __restrict__ tot, int64_t bpe,
                                                            int nparts, int64_t np) {
  const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= np) return;
  const int64_t c = g / nparts, x = g - c * nparts;
  int32_t* col = hist + c * bpe * nparts + x;
  int32_t run = 0;
  for (int64_t k0 = 0; k0 < bpe; k0 += 8) {
    int32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = k0 + u < bpe ? col[(k0 + u) * nparts] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (k0 + u < bpe) col[(k0 + u) * nparts] = run;
      run += v[u];
    }
  }
  tot[g] = run;
}

// one block: base[g] = exclusive prefix of tot over all partitions (epoch-major), base[np] = sum;
// base may alias tot
__global__ __launch_bounds__(1024) void csr_basescan_kernel(int32_t* tot, int32_t* base,
                                                            int64_t np) {
  __shared__ int32_t ws[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t per = (np + 1023) / 1024, a = tid * per, b = a + per < np ? a + per : np;
  int32_t s = 0;
  for (int64_t g = a; g < b; ++g) s += tot[g];
  int32_t inc = s;  // inclusive wave scan
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  int32_t run = inc - s;
  for (int w = 0; w < wave; ++w) run += ws[w];
  __syncthreads();  // every thread has its sums: base may overwrite tot now
  for (int64_t g = a; g < b; ++g) {
    const int32_t v = tot[g];
    base[g] = run;
    run += v;
  }
  if (tid == 1023) base[np] = run;
}

// The scattered (step id, position in partition) pairs: two arrays, or one 8-B word per step
// (packed: id | position << 32) where the scratch allows -- the scatter is bound by its store
// requests (configs[4]: 1.07 ms with two stores per step, 0.49 ms with one packed store;
// tools/csr_bench.py ablations)
struct Pairs {
  int32_t* id = nullptr;
  uint16_t* pos = nullptr;
  unsigned long long* pk = nullptr;
  __device__ __forceinline__ void get(int64_t e, int32_t& i, int32_t& p) const {
    if (pk) {
      const unsigned long long w = pk[e];
      i = (int32_t)(uint32_t)w;
      p = (int32_t)(w >> 32);
    } else {
      i = id[e];
      p = pos[e];
    }
  }
  __device__ __forceinline__ int32_t pos_of(int64_t e) const {
    return pk ? (int32_t)(pk[e] >> 32) : (int32_t)pos[e];
  }
  __device__ __forceinline__ void put(int64_t e, int32_t i, int32_t p) const {
    if (pk) {
      pk[e] = (unsigned long long)(uint32_t)i | ((unsigned long long)(uint32_t)p << 32);
    } else {
      id[e] = i;
      pos[e] = (uint16_t)p;
    }
  }
};

__global__ __launch_bounds__(kBlock) void csr_scatter_kernel(
    const int32_t* __restrict__ tgt, const int32_t* __restrict__ hist,
    const int32_t* __restrict__ base, Pairs pr, int32_t* __restrict__ out, int64_t n, int64_t bpe,
    int logp, int nparts) {
  extern __shared__ int32_t cur[];  // [nparts]
  const int64_t c = blockIdx.x / bpe, k = blockIdx.x - c * bpe;
  const int32_t* row = hist + (int64_t)blockIdx.x * nparts;
  for (int x = threadIdx.x; x < nparts; x += kBlock) cur[x] = base[c * nparts + x] + row[x];
  __syncthreads();
  const int32_t* t = tgt + c * n;
  const int32_t pm = (1 << logp) - 1;
  const int64_t i0 = k * kCsrChunk, i1 = i0 + kCsrChunk < n ? i0 + kCsrChunk : n;
  for (int64_t ib = i0; ib < i1; ib += 8 * kBlock) {
    int32_t p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = ib + u * kBlock + threadIdx.x;
      p[u] = i < i1 ? t[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = ib + u * kBlock + threadIdx.x;
      if (i >= i1) continue;
      if (i > 0 && (uint32_t)p[u] <= (uint32_t)i) {
        pr.put(atomicAdd(&cur[p[u] >> logp], 1), (int32_t)i, p[u] & pm);
      } else if (i > 0 && out) {
        out[c * n + i] = -1;  // a target outside [0, i]: no successor (fy_solve_kernel: j_i)
      }
    }
  }
}

// Bucket ranges of partition g in LDS: cnt[p] = its entries targeting position x * P + p,
// st[p] = their start in the partition's sorted range (exclusive prefix of cnt); NT threads
template <int NT = kBlock>
__device__ void csr_ranges(const Pairs& pr, int64_t b0, int64_t b1, int P, int32_t* cnt,
                           int32_t* st, int32_t* ws) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int p = tid; p < P; p += NT) cnt[p] = 0;
  __syncthreads();
  for (int64_t e = b0 + tid; e < b1; e += NT) atomicAdd(&cnt[pr.pos_of(e)], 1);
  __syncthreads();
  const int per = P / NT;
  int32_t s = 0;
  for (int j = 0; j < per; ++j) s += cnt[tid * per + j];
  int32_t inc = s;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  int32_t run = inc - s;
  for (int w = 0; w < wave; ++w) run += ws[w];
  for (int j = 0; j < per; ++j) {
    st[tid * per + j] = run;
    run += cnt[tid * per + j];
  }
  __syncthreads();
}

// fill: the partition's step ids into ent[], bucket by bucket; off (if given: the value walk on
// the packed layout) = the bucket starts, as csr_index_kernel<true> writes them
__global__ __launch_bounds__(kBlock) void csr_fill_kernel(Pairs pr,
                                                         const int32_t* __restrict__ base,
                                                         int32_t* __restrict__ ent,
                                                         int32_t* __restrict__ off, int64_t n,
                                                         int logp, int nparts) {
  extern __shared__ int32_t s[];  // cnt[P], cur[P]
  __shared__ int32_t ws[kBlock / 64];
  const int P = 1 << logp;
  const int64_t g = blockIdx.x, c = g / nparts, x = g - c * nparts;
  const int64_t b0 = base[g], b1 = base[g + 1];
  csr_ranges(pr, b0, b1, P, s, s + P, ws);
  int32_t* cur = s + P;
  if (off) {
    for (int p = threadIdx.x; p < P; p += kBlock) {
      const int64_t q = x * P + p;
      if (q >= n) break;
      off[c * (n + 1) + q] = (int32_t)(b0 + cur[p]);
      if (q == n - 1) off[c * (n + 1) + n] = (int32_t)(b0 + cur[p] + s[p]);
    }
    __syncthreads();  // every start read before the fill moves cur
  }
  for (int64_t e = b0 + threadIdx.x; e < b1; e += kBlock) {
    int32_t i, p;
    pr.get(e, i, p);
    ent[b0 + atomicAdd(&cur[p], 1)] = i;
  }
}

// fill + index for the resolution: the partition's buckets sorted into LDS (LDS = true; a
// partition of more than `cap` steps -- the lowest few, whose positions have the largest buckets
// -- into its range of ent instead, which this block then reads back from its own cache), then
// per position q: M(q) = min{i > q in bucket q} into mq, and for every step v of the bucket
// succ(v) = the next larger step of the bucket into succ (fy_solve_kernel's input)
// M(q) and succ(v) for every step v of bucket q = b[0 .. m) (in LDS or memory; the steps are
// distinct and >= q).  Small buckets by a min scan per step (what random targets give: ~ln(n/q)
// steps); a larger one -- adversarial but valid targets, e.g. every j_i = 0, one bucket of n - 1
// steps -- is heap-sorted in place first, O(m log m) in this thread instead of O(m^2).  succ is
// the epoch's base; returns M(q) (-1: none).
__device__ __forceinline__ int32_t csr_bucket_links(int32_t* __restrict__ b, int32_t m, int64_t q,
                                                    int32_t* __restrict__ succ) {
  if (m <= 32) {
    int32_t mq = 0x7FFFFFFF;
    for (int32_t k = 0; k < m; ++k) {
      const int32_t v = b[k];
      mq = (v > q && v < mq) ? v : mq;
      int32_t nx = 0x7FFFFFFF;
      for (int32_t f = 0; f < m; ++f) {
        const int32_t w = b[f];
        nx = (w > v && w < nx) ? w : nx;
      }
      succ[v] = nx == 0x7FFFFFFF ? -1 : nx;
    }
    return mq == 0x7FFFFFFF ? -1 : mq;
  }
  auto sift = [&](int32_t r, int32_t end) {
    for (;;) {
      int32_t ch = 2 * r + 1;
      if (ch >= end) break;
      if (ch + 1 < end && b[ch + 1] > b[ch]) ++ch;
      if (b[r] >= b[ch]) break;
      const int32_t t = b[r];
      b[r] = b[ch];
      b[ch] = t;
      r = ch;
    }
  };
  for (int32_t r = m / 2 - 1; r >= 0; --r) sift(r, m);
  for (int32_t end = m - 1; end > 0; --end) {
    const int32_t t = b[0];
    b[0] = b[end];
    b[end] = t;
    sift(0, end);
  }
  for (int32_t k = 0; k < m; ++k) succ[b[k]] = k + 1 < m ? b[k + 1] : -1;
  return b[0] > q ? b[0] : (m > 1 ? b[1] : -1);
}

constexpr int kFillBlock = 1024;  // fill + index: 16 waves a workgroup (its 64 KB of LDS allow
                                  // two workgroups per CU: 32 waves to hide the pair reads)

template <bool LDS>
__device__ __forceinline__ void csr_fill_index_body(const Pairs& pr, int64_t b0, int64_t b1,
                                                    int32_t* __restrict__ el, const int32_t* cnt,
                                                    int32_t* cur, int32_t* __restrict__ mq,
                                                    int32_t* __restrict__ succ, int64_t n,
                                                    int64_t c, int64_t x, int P) {
  for (int64_t e = b0 + threadIdx.x; e < b1; e += kFillBlock) {
    int32_t i, p;
    pr.get(e, i, p);
    el[atomicAdd(&cur[p], 1)] = i;
  }
  __syncthreads();  // cur[p] is now the end of bucket p
  for (int p = threadIdx.x; p < P; p += kFillBlock) {
    const int64_t q = x * P + p;
    if (q >= n) break;
    const int32_t k1 = cur[p], k0 = k1 - cnt[p];
    mq[c * n + q] = csr_bucket_links(el + k0, k1 - k0, q, succ + c * n);
  }
}

__global__ __launch_bounds__(kFillBlock) void csr_fill_index_kernel(
    Pairs pr, const int32_t* __restrict__ base, int32_t* __restrict__ ent,
    int32_t* __restrict__ mq, int32_t* __restrict__ succ, int64_t n, int logp, int nparts,
    int cap) {
  extern __shared__ int32_t s[];  // cnt[P], cur[P], the partition's buckets [cap]
  __shared__ int32_t ws[kFillBlock / 64];
  const int P = 1 << logp;
  const int64_t g = blockIdx.x, c = g / nparts, x = g - c * nparts;
  const int64_t b0 = base[g], b1 = base[g + 1];
  csr_ranges<kFillBlock>(pr, b0, b1, P, s, s + P, ws);
  if (b1 - b0 <= cap)
    csr_fill_index_body<true>(pr, b0, b1, s + 2 * P, s, s + P, mq, succ, n, c, x, P);
  else
    csr_fill_index_body<false>(pr, b0, b1, ent + b0, s, s + P, mq, succ, n, c, x, P);
}

// index: per position q of the partition, M(q) = min{i > q : j_i = q} (-1 if none) into mq[c][q]
// (WALK = false), or the start of bucket q in ent into off[c][q] (off[c][n] = the epoch's end)
template <bool WALK>
__global__ __launch_bounds__(kBlock) void csr_index_kernel(Pairs pr,
                                                          const int32_t* __restrict__ base,
                                                          int32_t* __restrict__ ent,
                                                          int32_t* __restrict__ dst,
                                                          int32_t* __restrict__ succ, int64_t n,
                                                          int logp, int nparts) {
  extern __shared__ int32_t s[];  // cnt[P], st[P]
  __shared__ int32_t ws[kBlock / 64];
  const int P = 1 << logp;
  const int64_t g = blockIdx.x, c = g / nparts, x = g - c * nparts;
  const int64_t b0 = base[g], b1 = base[g + 1];
  csr_ranges(pr, b0, b1, P, s, s + P, ws);
  for (int p = threadIdx.x; p < P; p += kBlock) {
    const int64_t q = x * P + p;
    if (q >= n) break;
    const int64_t e0 = b0 + s[P + p], e1 = e0 + s[p];
    if (WALK) {
      dst[c * (n + 1) + q] = (int32_t)e0;
      if (q == n - 1) dst[c * (n + 1) + n] = (int32_t)e1;
    } else {
      // (succ: fy_solve_kernel's input, read from out)
      dst[c * n + q] = csr_bucket_links(ent + e0, (int32_t)(e1 - e0), q, succ + c * n);
    }
  }
}

// the value walk over the sorted buckets (walk_pos's steps; bucket q = ent[off[q] .. off[q + 1]))
__device__ __forceinline__ int32_t walk_pos_csr(const int32_t* __restrict__ tgt,
                                                const int32_t* __restrict__ ent,
                                                const int32_t* __restrict__ off, int64_t tb,
                                                int64_t ob, int32_t n, int32_t v) {
  int32_t q = v, bound = n;
  for (;;) {
    int32_t best = -1;
    const int32_t e1 = off[ob + q + 1];
    for (int32_t e = off[ob + q]; e < e1; ++e) {
      const int32_t it = ent[e];
      best = (it > q && it < bound && it > best) ? it : best;
    }
    if (best >= 0 || q == 0) return best >= 0 ? best : 0;
    const int32_t jq = tgt[tb + q];
    if ((uint32_t)jq >= (uint32_t)q) return q;
    bound = q;
    q = jq;
  }
}

__global__ __launch_bounds__(kBlock) void csr_walk_scatter_kernel(const int32_t* __restrict__ tgt,
                                                                 const int32_t* __restrict__ ent,
                                                                 const int32_t* __restrict__ off,
                                                                 int32_t* __restrict__ perms,
                                                                 int64_t n, int64_t total) {
  for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < total;
       g += (int64_t)gridDim.x * kBlock) {
    const int64_t c = g / n;
    const int32_t v = (int32_t)(g - c * n);
    perms[c * n + walk_pos_csr(tgt, ent, off, c * n, c * (n + 1), (int32_t)n, v)] = v;
  }
}

__global__ __launch_bounds__(kBlock) void csr_walk_mark_kernel(const int32_t* __restrict__ tgt,
                                                              const int32_t* __restrict__ ent,
                                                              const int32_t* __restrict__ off,
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
    marks[c * n + walk_pos_csr(tgt, ent, off, c * n, c * (n + 1), (int32_t)n, v)] = l;
  }
}

// The partitioned buckets' geometry and scratch regions (int32 offsets) for count x n steps in
// `room` ints of scratch; ok = false: they do not fit (n too large for 4096 partitions of <= 4096
// positions, or tiny n) -- the linked lists run instead.  Two layouts:
//  * packed (the handle's scratch, perm_scratch_ints): 8-B pairs | ent | dst (M or the bucket
//    starts) | histograms | partition starts; the resolution then sorts each partition's buckets
//    in LDS and never writes them out (csr_fill_index_kernel);
//  * within the 3 * count * n the public dppo_perm_resolve documents: step ids (then dst) |
//    uint16 positions | ent | histograms | partition starts; fill and index are separate passes.
struct CsrPlan {
  bool ok = false, pack = false;
  int logp = 0, nparts = 0;
  int64_t bpe = 0, np = 0;
  int64_t r_id = 0, r_pos = 0, r_ent = 0, r_dst = 0, r_hist = 0, r_base = 0, end = 0;
};

CsrPlan csr_plan(int64_t n, int64_t count, int64_t room) {
  CsrPlan p;
  static const bool on = [] {
    const char* e = std::getenv("DPPO_PERM_CSR");
    return !(e && e[0] == '0');
  }();
  if (!on || n < 2 || count < 1) return p;
  int logp = kCsrMinLogP;
  while (logp < kCsrMaxLogP && ((n + (1ll << logp) - 1) >> logp) > kCsrMaxParts) ++logp;
  const int64_t nparts = (n + (1ll << logp) - 1) >> logp;
  if (nparts > kCsrMaxParts) return p;
  const int64_t total = n * count;
  if (total >= 0x7FFFFFFF) return p;
  p.logp = logp;
  p.nparts = (int)nparts;
  p.bpe = (n + kCsrChunk - 1) / kCsrChunk;
  p.np = nparts * count;
  auto al = [](int64_t x) { return (x + 63) / 64 * 64; };  // 256-B aligned regions
  const int64_t tail = al(count * p.bpe * nparts) + al(p.np + 1);
  // packed
  p.pack = true;
  p.r_id = 0;
  p.r_ent = al(2 * (total + 1));
  p.r_dst = p.r_ent + al(total);
  p.r_hist = p.r_dst + al(total + count + 1);
  p.r_base = p.r_hist + al(count * p.bpe * nparts);
  p.end = p.r_hist + tail;
  if (p.end <= room) {
    p.ok = true;
    return p;
  }
  // two arrays, dst over the step ids
  p.pack = false;
  p.r_id = 0;
  p.r_dst = 0;
  p.r_pos = al(total + count + 1);
  p.r_ent = p.r_pos + al((total + 1) / 2);
  p.r_hist = p.r_ent + al(total);
  p.r_base = p.r_hist + al(count * p.bpe * nparts);
  p.end = p.r_hist + tail;
  p.ok = p.end <= room;
  return p;
}

int64_t csr_room(int64_t n, int64_t count) {  // the scratch of the packed layout
  const CsrPlan p = csr_plan(n, count, INT64_MAX);
  return p.ok ? p.end : 0;
}

Pairs csr_pairs(const CsrPlan& P, int32_t* scratch) {
  Pairs pr;
  if (P.pack) {
    pr.pk = (unsigned long long*)(scratch + P.r_id);
  } else {
    pr.id = scratch + P.r_id;
    pr.pos = (uint16_t*)(scratch + P.r_pos);
  }
  return pr;
}

// count, colscan, basescan, scatter, and (fill) the buckets in ent; out: the resolution's output,
// where a step whose target lies outside [0, i] gets no successor
int csr_buckets(const CsrPlan& P, const int32_t* tgt, int32_t* scratch, int32_t* out, int64_t n,
                int64_t count, bool fill, hipStream_t s) {
  int32_t* hist = scratch + P.r_hist;
  int32_t* base = scratch + P.r_base;
  const Pairs pr = csr_pairs(P, scratch);
  const unsigned nchunks = (unsigned)(count * P.bpe), nb = (unsigned)P.np;
  const size_t lds_parts = (size_t)P.nparts * sizeof(int32_t);
  const size_t lds_fill = 2 * ((size_t)1 << P.logp) * sizeof(int32_t);
  DPPO_LAUNCH(csr_count_kernel, dim3(nchunks), dim3(kBlock), lds_parts, s, tgt, hist, n, P.bpe,
              P.logp, P.nparts);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(csr_colscan_kernel, dim3((unsigned)((P.np + kBlock - 1) / kBlock)), dim3(kBlock), 0,
              s, hist, base, P.bpe, P.nparts, P.np);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(csr_basescan_kernel, dim3(1), dim3(1024), 0, s, base, base, P.np);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(csr_scatter_kernel, dim3(nchunks), dim3(kBlock), lds_parts, s, tgt, hist, base, pr,
              out, n, P.bpe, P.logp, P.nparts);
  DPPO_LAUNCH_CHECK();
  if (!fill) return DPPO_OK;
  DPPO_LAUNCH(csr_fill_kernel, dim3(nb), dim3(kBlock), lds_fill, s, pr, base, scratch + P.r_ent,
              P.pack ? scratch + P.r_dst : nullptr, n, P.logp, P.nparts);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

// resolution (whole permutations) through the partitioned buckets
int csr_resolve(const CsrPlan& P, const int32_t* tgt, int32_t* perms, int32_t* scratch, int64_t n,
                int64_t count, bool walk, hipStream_t s) {
  {
    const int rc =
        csr_buckets(P, tgt, scratch, walk ? nullptr : perms, n, count, walk || !P.pack, s);
    if (rc != DPPO_OK) return rc;
  }
  const Pairs pr = csr_pairs(P, scratch);
  const int32_t* base = scratch + P.r_base;
  int32_t* ent = scratch + P.r_ent;
  int32_t* dst = scratch + P.r_dst;  // M, or the bucket starts (over the consumed step ids)
  const unsigned nb = (unsigned)P.np;
  const size_t lds = 2 * ((size_t)1 << P.logp) * sizeof(int32_t);
  if (walk) {
    if (!P.pack) {  // (packed: the fill wrote the bucket starts)
      DPPO_LAUNCH(csr_index_kernel<true>, dim3(nb), dim3(kBlock), lds, s, pr, base, ent, dst,
                  nullptr, n, P.logp, P.nparts);
      DPPO_LAUNCH_CHECK();
    }
    DPPO_LAUNCH(csr_walk_scatter_kernel, dim3(fy_grid(n * count)), dim3(kBlock), 0, s, tgt, ent,
                dst, perms, n, n * count);
    DPPO_LAUNCH_CHECK();
    return DPPO_OK;
  }
  if (P.pack) {
    // 64 KB of LDS per workgroup: cnt, cur, and the partition's steps if they fit (a heavier
    // partition sorts them into its own range of ent)
    const size_t lds_max = 65536 - 64;  // (the kernel's static wave sums)
    const int cap = (int)(lds_max / sizeof(int32_t)) - (2 << P.logp);
    DPPO_LAUNCH(csr_fill_index_kernel, dim3(nb), dim3(kFillBlock), lds_max, s, pr, base, ent, dst,
                perms, n, P.logp, P.nparts, cap);
    DPPO_LAUNCH_CHECK();
  } else {
    DPPO_LAUNCH(csr_index_kernel<false>, dim3(nb), dim3(kBlock), lds, s, pr, base, ent, dst,
                perms, n, P.logp, P.nparts);
    DPPO_LAUNCH_CHECK();
  }
  DPPO_LAUNCH(fy_solve_kernel, dim3(fy_grid(n * count)), dim3(kBlock), 0, s, tgt, dst, perms, n,
              n * count);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
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

int64_t perm_scratch_ints(int64_t n, int32_t count) {
  const int64_t r = csr_room(n, count);
  return r > 3 * n * (int64_t)count ? r : 3 * n * (int64_t)count;
}

int launch_perm_resolve(const int32_t* targets, int32_t* perms, int64_t n, int32_t count,
                        int32_t* scratch, int64_t scratch_ints, hipStream_t s) {
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
  {
    const CsrPlan P = csr_plan(n, count, scratch_ints);
    if (P.ok) return csr_resolve(P, targets, perms, scratch, n, count, perm_walk_env(false), s);
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
                                int64_t scratch_ints, int32_t* local, int32_t* seg, int32_t* cnt,
                                int64_t bg, int32_t ng, int32_t env0, int32_t nl, int32_t E,
                                int32_t M, hipStream_t s) {
  if (bg <= 0 || E <= 0) return DPPO_OK;
  const int64_t total = bg * E;
  const int64_t b_local = (bg / ng) * nl;
  DPPO_HIP_CHECK(hipMemsetAsync(marks, 0xFF, (size_t)total * sizeof(int32_t), s));
  const CsrPlan P = csr_plan(bg, E, scratch_ints);
  if (P.ok) {
    const int rc = csr_buckets(P, targets, scratch, nullptr, bg, E, true, s);
    if (rc != DPPO_OK) return rc;
    int32_t* off = scratch + P.r_dst;
    if (!P.pack) {  // (packed: the fill wrote the bucket starts)
      DPPO_LAUNCH(csr_index_kernel<true>, dim3((unsigned)P.np), dim3(kBlock),
                  2 * ((size_t)1 << P.logp) * sizeof(int32_t), s, csr_pairs(P, scratch),
                  scratch + P.r_base, scratch + P.r_ent, off, nullptr, bg, P.logp, P.nparts);
      DPPO_LAUNCH_CHECK();
    }
    DPPO_LAUNCH(csr_walk_mark_kernel, dim3(fy_grid(b_local * E)), dim3(kBlock), 0, s, targets,
                scratch + P.r_ent, off, marks, bg, b_local, E, ng, env0, nl);
    DPPO_LAUNCH_CHECK();
  } else {
    int32_t* head = scratch;
    int32_t* nxt = scratch + total;
    DPPO_HIP_CHECK(hipMemsetAsync(head, 0xFF, (size_t)total * sizeof(int32_t), s));
    DPPO_LAUNCH(fy_build_kernel, dim3(fy_grid(total)), dim3(kBlock), 0, s, targets, head, nxt, bg,
                total);
    DPPO_LAUNCH_CHECK();
    DPPO_LAUNCH(fy_walk_mark_kernel, dim3(fy_grid(b_local * E)), dim3(kBlock), 0, s, targets,
                head, nxt, marks, bg, b_local, E, ng, env0, nl);
    DPPO_LAUNCH_CHECK();
  }
  const dim3 grid((unsigned)shard_select_chunks(bg), (unsigned)E);
  DPPO_LAUNCH(shard_count_kernel<true>, grid, dim3(kBlock), 0, s, marks, cnt, bg, ng, env0, nl);
  DPPO_LAUNCH_CHECK();
  DPPO_LAUNCH(shard_write_kernel<true>, grid, dim3(kBlock), 0, s, marks, cnt, local, seg, bg, ng,
              env0, nl, M);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
