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

#include <cstdint>
#include <cstring>

#include "dppo_host.h"

namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908B0DFu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7FFFFFFFu;

struct MT {
  uint32_t mt[kN];
  int pos;
  uint32_t out[kN];  // tempered outputs of the current twist
  int opos;          // next index into out[]

  void twist() {
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
    pos = 0;
    opos = 0;
  }

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
    opos = p;
  }

  inline uint32_t next32() {
    if (opos >= kN) twist();
    ++pos;
    return out[opos++];
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

}  // namespace

extern "C" int dppo_perm_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                               int32_t* out) {
  if (!key || !pos || !out || n < 0 || n > 0x7FFFFFFF || count < 0 || *pos < 0 || *pos > kN)
    return DPPO_EINVAL;
  MT g;
  g.load(key, *pos);
  // Pass 1 draws the Fisher-Yates targets j[i] with a branch-free accept step (the draw is
  // always stored; i only advances on acceptance), pass 2 applies the swaps with the target
  // lines prefetched ahead -- the two passes are the same state machine as numpy's fused loop.
  uint32_t* j = new uint32_t[n > 1 ? n : 1];
  for (int32_t c = 0; c < count; ++c) {
    int32_t* a = out + (int64_t)c * n;
    for (int64_t k = 0; k < n; ++k) a[k] = (int32_t)k;
    int64_t i = n - 1;
    while (i >= 1) {
      const uint32_t mx = (uint32_t)i;
      const uint32_t mask = smear(mx);
      // all draws in [lo, i] share this mask
      const int64_t lo = (int64_t)((mask >> 1) + 1) > 1 ? (int64_t)((mask >> 1) + 1) : 1;
      while (i >= lo) {
        if (g.opos >= kN) g.twist();
        const uint32_t v = g.out[g.opos++] & mask;
        ++g.pos;
        j[i] = v;
        i -= (v <= (uint32_t)i) ? 1 : 0;
      }
    }
    constexpr int kAhead = 16;
    for (int64_t k = n - 1; k >= 1; --k) {
      if (k - kAhead >= 1) __builtin_prefetch(a + j[k - kAhead], 1, 3);
      const uint32_t v = j[k];
      const int32_t t = a[k];
      a[k] = a[v];
      a[v] = t;
    }
  }
  delete[] j;
  std::memcpy(key, g.mt, sizeof(g.mt));
  *pos = g.pos;
  return DPPO_OK;
}
