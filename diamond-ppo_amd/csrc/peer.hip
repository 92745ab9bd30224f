// Peer exchange: a one-shot all-reduce over directly mapped peer memory.
//
// The data-parallel learn sums two things over ranks (capi.cpp allreduce): the advantage
// statistics once per learn (2 doubles) and the gradient + loss partials once per minibatch
// (P + 8 floats, 52 KB for the default network) -- 33 dependent exchanges per learn, each on the
// critical path between a minibatch's gradient and its Adam step.  At 52 KB the exchange is pure
// latency, and on one MI355X node every GPU has a direct xGMI link to every other, so instead of a
// ring (RCCL: 2(W-1) dependent hops) every rank publishes its vector in its own exchange buffer
// and reads all W buffers at once, summing them in rank order 0..W-1 -- the same bits on every
// rank, and one link latency instead of 2(W-1).
//
// Buffer of each rank (hipMalloc, exported with hipIpcGetMemHandle, mapped by every peer; layout
// in common.h):  [values, 2 parities][tagged words, 2 parities][slice flags]
// Exchange `seq` (1, 2, ... the same sequence on every rank) uses parity seq & 1.  Workgroup s
// owns elements [s * kPeerChunk, (s + 1) * kPeerChunk): it copies its slice of the local vector
// into this rank's buffer, writes it back to memory (system-scope release: a peer reads our HBM
// over xGMI, not our L2), stores `seq` into its slice flag, then waits for flag s of every rank to
// reach `seq` (system-scope acquire) and sums the slice over ranks into the destination.
// Two parities suffice: a rank writes parity p again at exchange seq + 2 only after finishing
// exchange seq + 1, which waited for every peer's seq + 1 flags, which each peer set only after
// its own exchange seq -- its reads of parity p -- had completed (stream order).
//
// Memory ordering without cache maintenance: the slice is written with system-scope (sc0 sc1)
// stores -- coherent at system scope on their own, no L2 write-back of everything else dirty --
// drained with s_waitcnt vmcnt(0) before the flag store; the peers' slices are read with
// system-scope loads issued only after their flags were seen (in-order issue behind the poll's
// wait), so no L2 invalidate either.  (Measured against the fence-based form -- release/acquire
// fences, i.e. buffer_wbl2 / buffer_inv around plain accesses -- with 2 / 4 processes on one GPU:
// 6.0 / 6.7 us per 52 KB exchange against 8.0 / 13.7 us.)
//
// Waits are bounded (s_memrealtime) and checked against the handle's sticky error word: a rank
// that never arrives sets kErrPeerTimeout and every later wait gives up at once, so the grid
// always drains.
#include <hip/hip_runtime.h>

#include "common.h"

namespace dppo {
namespace {

constexpr int kPeerThreads = 256;

template <typename T>
__global__ __launch_bounds__(kPeerThreads) void peer_sum_kernel(PeerArgs a) {
  const int s = blockIdx.x;
  const int64_t i0 = (int64_t)s * kPeerChunk;
  const int64_t i1 = i0 + kPeerChunk < a.n ? i0 + kPeerChunk : a.n;
  const int64_t off = (int64_t)(a.seq & 1u) * a.data_bytes;
  T* mine = (T*)(a.bufs[a.rank] + off);
  const T* src = (const T*)a.src;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += kPeerThreads) peer_put(mine + i, src[i]);
  // every thread's slice stores are complete at system scope before the flag
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int failed;
  if (threadIdx.x == 0) {
    failed = 0;
    __hip_atomic_store(peer_flag(a, a.rank, s), a.seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  // thread r waits for rank r's flag of this slice
  if ((int)threadIdx.x < a.world && !peer_wait(peer_flag(a, threadIdx.x, s), a, threadIdx.x, s)) failed = 1;
  __syncthreads();
  if (failed) return;  // the destination keeps the local vector; the handle reports the error
  // every load of the thread's elements in flight before the first add (one link latency, not
  // one per element)
  constexpr int kPer = kPeerChunk / kPeerThreads;
  T v[kPer][kMaxPeers];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = i0 + threadIdx.x + k * kPeerThreads;
#pragma unroll
    for (int r = 0; r < kMaxPeers; ++r)
      v[k][r] = (r < a.world && i < i1) ? peer_get((const T*)(a.bufs[r] + off) + i) : T(0);
  }
  T* dst = (T*)a.dst;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = i0 + threadIdx.x + k * kPeerThreads;
    T acc = v[k][0];
#pragma unroll
    for (int r = 1; r < kMaxPeers; ++r)
      if (r < a.world) acc += v[k][r];
    if (i < i1) dst[i] = acc;
  }
}

}  // namespace

int64_t peer_buffer_bytes(int64_t cap) { return 4 * cap * 8 + 64 * (int64_t)kPeerMaxSlices; }

int launch_peer_sum(const PeerArgs& a, bool f64, hipStream_t s) {
  const int64_t g = (a.n + kPeerChunk - 1) / kPeerChunk;
  if (a.n < 1 || g > kPeerMaxSlices || a.world < 1 || a.world > kMaxPeers || a.rank < 0 ||
      a.rank >= a.world || a.n * (f64 ? 8 : 4) > a.data_bytes) {
    set_error("peer exchange of %lld elements does not fit the exchange buffer", (long long)a.n);
    return DPPO_EINVAL;
  }
  if (f64)
    DPPO_LAUNCH(peer_sum_kernel<double>, dim3((unsigned)g), dim3(kPeerThreads), 0, s, a);
  else
    DPPO_LAUNCH(peer_sum_kernel<float>, dim3((unsigned)g), dim3(kPeerThreads), 0, s, a);
  DPPO_LAUNCH_CHECK();
  return DPPO_OK;
}

}  // namespace dppo
