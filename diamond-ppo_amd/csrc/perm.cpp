// Host-side minibatch permutations, bit-exact with NumPy's legacy RandomState.permutation.
//
// The reference draws its minibatch order from the legacy global NumPy RNG
// (diamond/ppo.py:120-122 seeds it; ppo.py:254 calls np.random.permutation(batch_size) once per
// epoch).  NumPy's algorithm (numpy 2.2.6, restated in oracle/mt19937.py):
//   permutation(n) = arange(n) shuffled by Fisher-Yates, i = n-1 .. 1,
//   j = random_interval(i) = (next_uint32 & mask) redrawn until <= i (mask = 2^k-1 >= i),
//   next_uint32 = MT19937 genrand_int32 (624-word twist + tempering).
// We run the same state machine on the caller's MT19937 key/pos (taken from
// np.random.get_state()) and hand the advanced key/pos back, so the global NumPy RNG ends
// exactly where the reference leaves it.  Output is int32 (B < 2^31), ready for upload.
//
// Throughput: the twist is written so the compiler vectorises it; the draw/accept loop is
// branch-light; the swap runs on a 4-byte array (2 MiB at B = 524,288 fits in L2).
// dppo_perm_targets_numpy stops after the draws: the swaps are resolved on the GPU instead
// (shuffle.hip), which takes the sequential swap chain off the host's critical path.

#include <immintrin.h>

#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "dppo_host.h"

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908B0DFu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7FFFFFFFu;

// One MT19937 block: twist the 624-word state and temper it into out[].  The three twist
// ranges only depend on words at distance >= 227 (or the block before), so each loop
// vectorises; AVX2 clones are picked at load time where the host has them.
__attribute__((target_clones("avx512f", "avx2", "default"))) void twist_block(uint32_t* __restrict mt,
                                                                   uint32_t* __restrict out) {
  int i = 0;
  for (; i < kN - kM; ++i) {
    uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  for (; i < kN - 1; ++i) {
    uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  uint32_t y = (mt[kN - 1] & kUpper) | (mt[0] & kLower);
  mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  for (int k = 0; k < kN; ++k) {
    uint32_t t = mt[k];
    t ^= t >> 11;
    t ^= (t << 7) & 0x9D2C5680u;
    t ^= (t << 15) & 0xEFC60000u;
    t ^= t >> 18;
    out[k] = t;
  }
}

struct MT {
  uint32_t mt[kN];
  uint32_t out[kN];  // tempered outputs of the current block
  int pos;           // next unconsumed word of the block (numpy's `pos`)

  void load(const uint32_t* key, int p) {
    std::memcpy(mt, key, sizeof(mt));
    pos = p;
    // Words [p, 624) of the current block are still unconsumed: temper them now.
    for (int k = p; k < kN; ++k) {
      uint32_t t = mt[k];
      t ^= t >> 11;
      t ^= (t << 7) & 0x9D2C5680u;
      t ^= (t << 15) & 0xEFC60000u;
      t ^= t >> 18;
      out[k] = t;
    }
  }
};

inline uint32_t smear(uint32_t m) {
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  m |= m >> 8;
  m |= m >> 16;
  return m;
}

// AVX-512 draws, 16 per step.  Inside a mask band a draw is accepted iff v <= i, and i falls by
// at most one per draw, so over a group of 16 draws starting at i every v <= i - 15 is accepted
// and every v > i rejected whatever the others do: the group's outcome needs no serial chain
// unless some v lands in (i - 15, i].  The accepted draws, in order, are the targets j[i],
// j[i-1], ...: one compress, one reversal, one masked store.  Returns the words consumed; stops
// at the first ambiguous group, when i < lo + 15 (the band's last draws) or at the block end.
__attribute__((target("avx512f,avx512vl"))) uint32_t draw_groups_avx512(const uint32_t* o,
                                                                         uint32_t words,
                                                                         uint32_t mask, uint32_t& i,
                                                                         uint32_t lo, int32_t* j) {
  const __m512i vmask = _mm512_set1_epi32((int)mask);
  const __m512i rev = _mm512_set_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  uint32_t k = 0;
  uint32_t ii = i;
  while (k + 16 <= words && ii >= lo + 15) {
    const __m512i v = _mm512_and_si512(_mm512_loadu_si512((const void*)(o + k)), vmask);
    const __mmask16 acc = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)(ii - 15)));
    const __mmask16 amb =
        (__mmask16)(_mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)ii)) & ~acc);
    if (amb) break;
    const int cnt = __builtin_popcount((unsigned)acc);
    const __m512i c = _mm512_maskz_compress_epi32(acc, v);
    const __m512i r = _mm512_permutexvar_epi32(rev, c);
    _mm512_mask_storeu_epi32((void*)(j + (int64_t)ii - 15), (__mmask16)(0xFFFFu << (16 - cnt)),
                             r);
    ii -= (uint32_t)cnt;
    k += 16;
  }
  i = ii;
  return k;
}

bool has_avx512() {
  static const bool yes = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl");
  return yes;
}

// Fisher-Yates targets of `count` successive permutations of arange(n): j[c][i] for
// i = n-1 .. 1 (j[c][0] = 0), the draw/accept state machine of numpy's random_interval with the
// accept step branch-free (the draw is always stored; i only advances on acceptance).
// Within one mask band [lo, i] the loop runs min(words left in the block, i - lo + 1) draws
// with no exit test: i falls by at most one per draw, so it cannot leave the band early.
void draw_targets(MT& g, int64_t n, int32_t count, int32_t* __restrict out) {
  int opos = g.pos;
  const bool simd = has_avx512();
  for (int32_t c = 0; c < count; ++c) {
    int32_t* __restrict j = out + (int64_t)c * n;
    if (n > 0) j[0] = 0;
    uint32_t i = n > 0 ? (uint32_t)(n - 1) : 0u;
    while (i >= 1) {
      const uint32_t mask = smear(i);
      const uint32_t lo = (mask >> 1) + 1;  // all draws in [lo, i] share this mask
      while (i >= lo) {
        if (opos >= kN) {
          twist_block(g.mt, g.out);
          opos = 0;
        }
        if (simd && i >= lo + 15) {
          opos += (int)draw_groups_avx512(g.out + opos, (uint32_t)(kN - opos), mask, i, lo, j);
          if (opos >= kN || i < lo) continue;
        }
        const uint32_t* __restrict o = g.out + opos;
        const uint32_t left = (uint32_t)(kN - opos);
        uint32_t run = left < i - lo + 1 ? left : i - lo + 1;
        if (simd && run > 16) run = 16;  // one group by the serial chain, then SIMD again
        for (uint32_t k = 0; k < run; ++k) {
          const uint32_t v = o[k] & mask;
          j[i] = (int32_t)v;
          // accept (v <= i): i - 1; reject: i.  cmp sets CF = (i < v), adc adds CF - 1: a
          // 2-cycle loop-carried chain instead of the compiler's cmp/setcc/movzx/sub
#if defined(__x86_64__)
          asm("cmpl %1, %0\n\tadcl $-1, %0" : "+r"(i) : "r"(v) : "cc");
#else
          i = i - 1u + (i < v ? 1u : 0u);
#endif
        }
        opos += (int)run;
      }
    }
  }
  g.pos = opos;
}

// a[0..n) holds Fisher-Yates targets on entry and the permutation on exit: the sequential
// swap loop for i = n-1 .. 1, with the target lines prefetched ahead.
void apply_swaps(int32_t* a, int64_t n) {
  std::vector<int32_t> j(a, a + n);
  for (int64_t k = 0; k < n; ++k) a[k] = (int32_t)k;
  constexpr int kAhead = 16;
  for (int64_t k = n - 1; k >= 1; --k) {
    if (k - kAhead >= 1) __builtin_prefetch(a + j[k - kAhead], 1, 3);
    const int32_t v = j[k];
    const int32_t t = a[k];
    a[k] = a[v];
    a[v] = t;
  }
}

bool bad_args(const uint32_t* key, const int32_t* pos, int64_t n, int32_t count,
              const int32_t* out) {
  return !key || !pos || !out || n < 0 || n > 0x7FFFFFFF || count < 0 || *pos < 0 || *pos > kN;
}

}  // namespace

extern "C" int dppo_perm_targets_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                                       int32_t* out) {
  if (bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  MT g;
  g.load(key, *pos);
  draw_targets(g, n, count, out);
  std::memcpy(key, g.mt, sizeof(g.mt));
  *pos = g.pos;
  return DPPO_OK;
}

extern "C" int dppo_perm_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                               int32_t* out) {
  if (bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  MT g;
  g.load(key, *pos);
  // Targets first (into out itself), then the swaps in place -- the same state machine as
  // numpy's fused loop.  The draws are one sequential MT19937 stream; the swaps of epoch c only
  // need epoch c's targets, so at minibatch sizes each epoch's swaps run on a worker thread
  // while the next epoch is drawn (wall ~ draws + one epoch's swaps).
  const bool threaded = n >= (1 << 16) && count > 1;
  std::vector<std::thread> workers;
  for (int32_t c = 0; c < count; ++c) {
    draw_targets(g, n, 1, out + (int64_t)c * n);
    if (threaded)
      workers.emplace_back(apply_swaps, out + (int64_t)c * n, n);
    else
      apply_swaps(out + (int64_t)c * n, n);
  }
  for (auto& w : workers) w.join();
  std::memcpy(key, g.mt, sizeof(g.mt));
  *pos = g.pos;
  return DPPO_OK;
}
