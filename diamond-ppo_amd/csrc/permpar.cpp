// Parallel, bit-exact draw of NumPy-legacy permutation targets.
//
// Reference: diamond/ppo.py:252-255 draws E permutations of the batch from the global legacy
// RandomState, np.random.permutation(B) once per epoch.  perm.cpp restates the draw serially:
// one MT19937 word stream consumed by an accept scan,
//     target k (epoch e = k / (n-1), index i = n-1 - k % (n-1)) = the first unconsumed word w
//     whose masked value v = w & smear(i) is <= i,
// which costs ~16-21 ms per learn at BASELINE configs[4] with global minibatches (4 x 8.4 M
// targets from ~46 M words) and capped the reference-exact multi-GPU mode at ~2x.  Where the
// scan stands at a given word (its counter k) depends on every accept and reject before it, so
// the stream cannot simply be cut among threads.  This file cuts it anyway:
//
// (1) Jump-ahead.  The word stream does not depend on the scan.  Chunk c (a run of whole MT19937
//     blocks) gets the generator state at its first block by evaluating g(x) = x^J mod phi(x)
//     at the one-word MT19937 transition F (Horner: 19,937 steps, each one word of F plus a
//     624-word XOR), phi = the characteristic polynomial of F, found once per process by
//     Berlekamp-Massey over 40 K output bits.  ~0.2 ms per chunk.
// (2) Speculation.  Every chunk is scanned by its own thread from a GUESSED counter: the
//     expected counter at its first word (acceptance probability (i+1)/(mask+1) per word).  The
//     guessed run is a genuine run of the scan, started from the wrong counter.
// (3) Exact correction (serial, a fraction of the words).  Two runs that read the same word with
//     counters k_t (true) and k_g (guess) in the same mask band have indices i_t = i_g + d,
//     d = k_g - k_t.  They agree on every word except one whose masked value lies in
//     (min(i_g, i_t), max(i_g, i_t)]: there exactly one of them accepts, and |d| shrinks by one.
//     So the true run's targets are the guessed run's targets shifted by d, with one insertion or
//     deletion per such word.  The guessed run records every word whose masked value lies within
//     W of its own index ("near misses": all the words that can disagree while |d| <= W).  The
//     two runs may use different masks only around a band change (powers of two, epoch ends, the
//     draw's end); around those the guessed run also keeps the raw words and its accept bits
//     ("zones": wherever its counter is within Wb of a band change), and the stitcher replays the
//     true run word by word exactly where the two runs sit in different bands.
// (4) Assembly (parallel): chunk c's true targets = copies of its guessed targets + literals.
// Any check that fails (|d| > W, a replay past the kept words, a missing key) falls back to the
// serial draw, so the result is always exact; dppo_perm_targets_numpy_par reports which path ran.
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "dppo_host.h"

// perm.cpp: the serial draw (the fallback, and the path for small draws)
int dppo_perm_targets_serial(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out);

namespace {

#define PAR_AVX512 __attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt,pclmul")))

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908B0DFu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7FFFFFFFu;

inline uint32_t temper1(uint32_t t) {
  t ^= t >> 11;
  t ^= (t << 7) & 0x9D2C5680u;
  t ^= (t << 15) & 0xEFC60000u;
  t ^= t >> 18;
  return t;
}

inline uint32_t smear(uint32_t m) {
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  m |= m >> 8;
  m |= m >> 16;
  return m;
}

PAR_AVX512 void twist_temper(uint32_t* __restrict mt, uint32_t* __restrict out) {
  int i = 0;
  for (; i < kN - kM; ++i) {
    const uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  for (; i < kN - 1; ++i) {
    const uint32_t y = (mt[i] & kUpper) | (mt[i + 1] & kLower);
    mt[i] = mt[i + (kM - kN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }
  const uint32_t y = (mt[kN - 1] & kUpper) | (mt[0] & kLower);
  mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  for (int k = 0; k < kN; ++k) out[k] = temper1(mt[k]);
}

// ------------------------------------------------------------------------------------------
// GF(2)[x] modulo phi, the characteristic polynomial of the MT19937 one-word transition
// ------------------------------------------------------------------------------------------
constexpr int kDeg = 19937;
constexpr int kPW = 312;  // 64-bit words of a polynomial of degree <= 19937
using Poly = std::vector<uint64_t>;

inline uint64_t get64(const uint64_t* p, int64_t off) {
  const int64_t w = off >> 6;
  const int b = (int)(off & 63);
  return b ? (p[w] >> b) | (p[w + 1] << (64 - b)) : p[w];
}

// p ^= q << sh (bit shift), q: nq words
inline void xor_shifted(uint64_t* p, const uint64_t* q, int nq, int64_t sh) {
  const int64_t ws = sh >> 6;
  const int bs = (int)(sh & 63);
  if (!bs) {
    for (int j = 0; j < nq; ++j) p[ws + j] ^= q[j];
    return;
  }
  for (int j = 0; j < nq; ++j) {
    p[ws + j] ^= q[j] << bs;
    p[ws + j + 1] ^= q[j] >> (64 - bs);
  }
}

// phi by Berlekamp-Massey over bit 0 of the untempered words x_624, x_625, ... of the generator
// seeded 5489 (MT19937's characteristic polynomial is primitive, so every non-zero output
// sequence has it as its minimal polynomial).
Poly berlekamp_massey_phi() {
  const int64_t NN = 2 * kDeg + 128;
  std::vector<uint32_t> mt(kN), tmp(kN);
  mt[0] = 5489u;
  for (int i = 1; i < kN; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  const int64_t rw = (2 * NN) / 64 + 8;
  std::vector<uint64_t> R(rw, 0);  // reversed sequence: bit j = s[NN-1-j]
  for (int64_t k = 0; k < NN;) {
    twist_temper(mt.data(), tmp.data());
    for (int j = 0; j < kN && k < NN; ++j, ++k)
      if (mt[j] & 1u) {
        const int64_t b = NN - 1 - k;
        R[b >> 6] |= 1ull << (b & 63);
      }
  }
  const int cw = (int)(NN / 64) + 8;
  std::vector<uint64_t> C(cw, 0), B(cw, 0), T(cw, 0);
  C[0] = B[0] = 1;
  int64_t L = 0, m = 1;
  for (int64_t n = 0; n < NN; ++n) {
    const int64_t base = NN - 1 - n;  // s[n-i] = R bit (base + i)
    uint64_t acc = 0;
    const int wmax = (int)(L >> 6);
    for (int w = 0; w <= wmax; ++w) acc ^= C[w] & get64(R.data(), base + 64 * (int64_t)w);
    if (!__builtin_parityll(acc)) {
      ++m;
      continue;
    }
    const int nb = (int)((n + 1) / 64) + 2;  // B's degree < n + 1
    if (2 * L <= n) {
      T = C;
      xor_shifted(C.data(), B.data(), std::min(nb, cw - (int)(m >> 6) - 2), m);
      L = n + 1 - L;
      B.swap(T);
      m = 1;
    } else {
      xor_shifted(C.data(), B.data(), std::min(nb, cw - (int)(m >> 6) - 2), m);
      ++m;
    }
  }
  if (L != kDeg) return Poly();
  Poly phi(kPW, 0);  // phi(x) = x^L C(1/x)
  for (int64_t i = 0; i <= L; ++i)
    if ((C[i >> 6] >> (i & 63)) & 1) phi[(L - i) >> 6] |= 1ull << ((L - i) & 63);
  return phi;
}

struct Gf2 {
  Poly phi;
  std::vector<uint64_t> tab;  // tab[b * kPW ...] = (b(x) x^19937) mod phi, b < 256
  bool ok = false;

  void init() {
    phi = berlekamp_massey_phi();
    if (phi.empty()) return;
    tab.assign(256 * (size_t)kPW, 0);
    Poly t = phi;  // x^19937 = phi - x^19937 (mod phi)
    t[kDeg >> 6] &= ~(1ull << (kDeg & 63));
    std::vector<Poly> base(8);
    for (int j = 0; j < 8; ++j) {
      base[j] = t;
      t = mulx(t);
    }
    for (int b = 1; b < 256; ++b)
      for (int j = 0; j < 8; ++j)
        if (b & (1 << j))
          for (int w = 0; w < kPW; ++w) tab[(size_t)b * kPW + w] ^= base[j][w];
    ok = true;
  }

  Poly mulx(const Poly& a) const {
    Poly r(kPW, 0);
    for (int w = kPW - 1; w > 0; --w) r[w] = (a[w] << 1) | (a[w - 1] >> 63);
    r[0] = a[0] << 1;
    if ((r[kDeg >> 6] >> (kDeg & 63)) & 1)
      for (int w = 0; w < kPW; ++w) r[w] ^= phi[w];
    return r;
  }

  // p (>= 2*kPW + 2 words, degree <= top) -> p mod phi, 8 bits at a time from the top
  void reduce(uint64_t* p, int64_t top) const {
    if (top < kDeg) return;
    for (int64_t t = kDeg + ((top - kDeg) / 8) * 8; t >= kDeg; t -= 8) {
      const uint32_t byte = (uint32_t)(get64(p, t) & 0xFFu);
      if (!byte) continue;
      // clear the byte, add its residue
      const int64_t w = t >> 6;
      const int b = (int)(t & 63);
      p[w] &= ~(0xFFull << b);
      if (b > 56) p[w + 1] &= ~(0xFFull >> (64 - b));
      xor_shifted(p, tab.data() + (size_t)byte * kPW, kPW, t - kDeg);
    }
  }

  PAR_AVX512 Poly mulmod(const Poly& a, const Poly& b) const {
    std::vector<uint64_t> p(2 * kPW + 4, 0);
    for (int i = 0; i < kPW; ++i) {
      if (!a[i]) continue;
      const __m128i x = _mm_set_epi64x(0, (long long)a[i]);
      for (int j = 0; j < kPW; ++j) {
        const __m128i r = _mm_clmulepi64_si128(x, _mm_set_epi64x(0, (long long)b[j]), 0);
        p[i + j] ^= (uint64_t)_mm_cvtsi128_si64(r);
        p[i + j + 1] ^= (uint64_t)_mm_extract_epi64(r, 1);
      }
    }
    reduce(p.data(), 2 * (int64_t)kDeg);
    return Poly(p.begin(), p.begin() + kPW);
  }

  PAR_AVX512 Poly sqrmod(const Poly& a) const {
    std::vector<uint64_t> p(2 * kPW + 4, 0);
    for (int i = 0; i < kPW; ++i) {
      const __m128i x = _mm_set_epi64x(0, (long long)a[i]);
      const __m128i r = _mm_clmulepi64_si128(x, x, 0);
      p[2 * i] = (uint64_t)_mm_cvtsi128_si64(r);
      p[2 * i + 1] = (uint64_t)_mm_extract_epi64(r, 1);
    }
    reduce(p.data(), 2 * (int64_t)kDeg);
    return Poly(p.begin(), p.begin() + kPW);
  }

  Poly powx(uint64_t e) const {
    Poly r(kPW, 0);
    r[0] = 1;
    for (int b = e ? 63 - __builtin_clzll(e) : -1; b >= 0; --b) {
      r = sqrmod(r);
      if ((e >> b) & 1) r = mulx(r);
    }
    return r;
  }
};

const Gf2& field() {
  static Gf2 f;
  static std::once_flag once;
  std::call_once(once, [] { f.init(); });
  return f;
}

// r ^= t for a circular window r (element j at r[(off + j) % 624]) and a plain window t
PAR_AVX512 inline void xor_window(uint32_t* r, int off, const uint32_t* t) {
  const int a = kN - off;  // elements 0 .. a-1 at r[off ..], a .. 623 at r[0 ..]
  int j = 0;
  for (; j + 16 <= a; j += 16)
    _mm512_storeu_si512((void*)(r + off + j),
                        _mm512_xor_si512(_mm512_loadu_si512((const void*)(r + off + j)),
                                         _mm512_loadu_si512((const void*)(t + j))));
  for (; j < a; ++j) r[off + j] ^= t[j];
  int k = 0;  // r[k] ^= t[a + k], k < off
  for (; k + 16 <= off; k += 16)
    _mm512_storeu_si512((void*)(r + k),
                        _mm512_xor_si512(_mm512_loadu_si512((const void*)(r + k)),
                                         _mm512_loadu_si512((const void*)(t + a + k))));
  for (; k < off; ++k) r[k] ^= t[a + k];
}

// one word of the recurrence into the oldest slot of a circular window
inline int step_window(uint32_t* r, int off) {
  const int o1 = off + 1 == kN ? 0 : off + 1;
  const int oM = off + kM >= kN ? off + kM - kN : off + kM;
  const uint32_t y = (r[off] & kUpper) | (r[o1] & kLower);
  r[off] = r[oM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  return o1;
}

// out = the 624-word window g(F) s (window element j = x_{J + j}, lower 31 bits of element 0
// not determined).  Horner four coefficients at a time: r = F^4(r) ^ T[nibble], where
// T[m] = sum of F^j s over the bits j of m (16 precomputed windows).
PAR_AVX512 void jump_window(const uint32_t* s, const Poly& g, uint32_t* out) {
  std::vector<uint32_t> tab(16 * (size_t)kN, 0);
  {
    alignas(64) uint32_t w[kN];
    std::memcpy(w, s, sizeof(w));
    int off = 0;
    for (int j = 0; j < 4; ++j) {  // F^j s, in window order
      uint32_t* fj = tab.data() + (size_t)(1 << j) * kN;
      for (int e = 0; e < kN; ++e) fj[e] = w[(off + e) % kN];
      off = step_window(w, off);
    }
    for (int m = 1; m < 16; ++m) {
      if ((m & (m - 1)) == 0) continue;
      uint32_t* t = tab.data() + (size_t)m * kN;
      const uint32_t* lo = tab.data() + (size_t)(m & -m) * kN;
      const uint32_t* rest = tab.data() + (size_t)(m & (m - 1)) * kN;
      for (int e = 0; e < kN; ++e) t[e] = lo[e] ^ rest[e];
    }
  }
  alignas(64) uint32_t r[kN];
  std::memset(r, 0, sizeof(r));
  int off = 0;
  int deg = kPW * 64 - 1;
  while (deg >= 0 && !((g[deg >> 6] >> (deg & 63)) & 1)) --deg;
  const int top = deg < 0 ? -1 : deg / 4;
  for (int t = top; t >= 0; --t) {
    if (t != top)
      for (int j = 0; j < 4; ++j) off = step_window(r, off);
    const int nib = (int)((g[(4 * t) >> 6] >> ((4 * t) & 63)) & 15);
    if (nib) xor_window(r, off, tab.data() + (size_t)nib * kN);
  }
  for (int j = 0; j < kN; ++j) out[j] = r[(off + j) % kN];
}

// The key (untempered words) of block `blocks` after the block whose key is key0:
// window at sliding index 624*blocks - 1, then one more step.
struct JumpCache {
  std::mutex mu;
  std::map<uint64_t, Poly> polys;
  Poly get(uint64_t e) {
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = polys.find(e);
      if (it != polys.end()) return it->second;
    }
    Poly p = field().powx(e);
    std::lock_guard<std::mutex> g(mu);
    if (polys.size() > 256) polys.clear();
    polys[e] = p;
    return p;
  }
};
JumpCache& jump_cache() {
  static JumpCache* c = new JumpCache();
  return *c;
}

void key_after_blocks(const uint32_t* key0, int64_t blocks, uint32_t* key) {
  alignas(64) uint32_t w[kN];
  const Poly g = jump_cache().get((uint64_t)(kN * blocks - 1));
  jump_window(key0, g, w);
  // one more step: window at 624*blocks = x_{624 b} .. x_{624 b + 623}, every word exact
  const uint32_t y = (w[0] & kUpper) | (w[1] & kLower);
  const uint32_t nw = w[kM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  std::memcpy(key, w + 1, (kN - 1) * sizeof(uint32_t));
  key[kN - 1] = nw;
}

// ------------------------------------------------------------------------------------------
// The expected-counter model: acceptance probability (i+1)/(mask+1) per word
// ------------------------------------------------------------------------------------------
double harm(double m) {  // H(m) = sum_{j<=m} 1/j
  if (m < 64) {
    double s = 0;
    for (int j = 1; j <= (int)m; ++j) s += 1.0 / j;
    return s;
  }
  const double i2 = 1.0 / (m * m);
  return std::log(m) + 0.57721566490153286 + 0.5 / m - i2 / 12.0 + i2 * i2 / 120.0;
}
double harm2(double m) {  // sum_{j<=m} 1/j^2
  if (m < 64) {
    double s = 0;
    for (int j = 1; j <= (int)m; ++j) s += 1.0 / ((double)j * j);
    return s;
  }
  return 1.6449340668482264 - (1.0 / m - 0.5 / (m * m) + 1.0 / (6.0 * m * m * m));
}

struct Model {
  int64_t n = 0, count = 0, K = 0;  // K = count * (n - 1) targets
  struct Seg {
    int64_t k0, k1, ihi;
    double M, E0, V0;  // expected words / word variance before k0 (within the epoch)
  };
  std::vector<Seg> segs;  // one epoch
  double E_ep = 0, V_ep = 0;

  void init(int64_t n_, int64_t count_) {
    n = n_;
    count = count_;
    K = count * (n - 1);
    segs.clear();
    double E = 0, V = 0;
    int64_t k = 0;
    for (int64_t ihi = n - 1; ihi >= 1;) {
      const uint32_t mask = smear((uint32_t)ihi);
      const int64_t lo = (mask >> 1) + 1;
      const double M = (double)mask + 1.0;
      Seg s{k, k + (ihi - lo + 1), ihi, M, E, V};
      segs.push_back(s);
      E += M * (harm((double)ihi + 1) - harm((double)lo));
      V += M * M * (harm2((double)ihi + 1) - harm2((double)lo)) -
           M * (harm((double)ihi + 1) - harm((double)lo));
      k = s.k1;
      ihi = lo - 1;
    }
    E_ep = E;
    V_ep = V;
  }
  // expected words / word variance to draw targets [0, k)
  void before(int64_t k, double* E, double* V) const {
    if (k >= K) k = K;
    const int64_t e = k / (n - 1);
    const int64_t r = k - e * (n - 1);
    double e0 = E_ep * (double)e, v0 = V_ep * (double)e;
    const Seg* s = &segs[0];
    for (const Seg& t : segs)
      if (t.k0 <= r) s = &t;
    const double a = (double)s->ihi + 1, b = (double)(s->ihi - (r - s->k0)) + 1;
    *E = e0 + s->E0 + s->M * (harm(a) - harm(b));
    *V = v0 + s->V0 + s->M * s->M * (harm2(a) - harm2(b)) - s->M * (harm(a) - harm(b));
  }
  // G(w): the counter whose expected word count is closest to w
  int64_t counter_at(double w) const {
    int64_t lo = 0, hi = K;
    while (lo < hi) {
      const int64_t mid = lo + (hi - lo) / 2;
      double E, V;
      before(mid, &E, &V);
      if (E < w) lo = mid + 1;
      else hi = mid;
    }
    return lo;
  }
};

// ------------------------------------------------------------------------------------------
// Speculative chunk scans
// ------------------------------------------------------------------------------------------
struct Zone {  // words [q0, q1) kept: raw[raw0 + ..], accept bit (raw0 + ..) of bits
  uint32_t q0, q1;
  int64_t raw0;
  int64_t k0;  // guessed counter at q0
};
struct Op {  // true targets [k, k + len): guessed targets S[src ..] or literals L[src ..]
  int64_t k;
  int64_t src;
  int64_t len;
  int32_t lit;
};

struct Chunk {
  // inputs
  int64_t Q0 = 0;        // global word index of the first word
  int64_t len = 0;       // words (last chunk: open-ended, -1)
  int64_t block0 = 0;    // block of the first word
  int32_t off0 = 0;      // word offset in block0
  int64_t kg0 = 0;       // guessed counter at the first word
  // outputs of the scan
  std::vector<int32_t> S;  // guessed targets k = kg0 ..
  // near misses (structure of arrays, sorted by q): word, guessed targets before it,
  // masked value - guessed index, masked value
  std::vector<uint32_t> rq, rs, rm;
  std::vector<int32_t> ru;
  int64_t W = 0, Wb = 0;  // near-miss band and zone half-width (counter units) of this chunk
  std::vector<std::pair<int64_t, int64_t>> zone_iv;  // merged [lo, hi] guessed-counter intervals
  std::vector<Zone> zones;
  std::vector<uint32_t> raw;       // kept words (nraw used)
  std::vector<uint64_t> bits;      // their accept bits, packed
  std::vector<uint32_t> pref;      // accepts in raw[0 .. 64 b)
  int64_t nraw = 0;
  std::vector<int64_t> key_blocks;  // keys of the blocks near the draw's end
  std::vector<uint32_t> keys;
  int64_t words = 0, kg_end = 0, q_done = -1, ns = 0;
  bool overflow = false;
  double us = 0, jump_us = 0;
  int64_t scalar_words = 0;
  uint64_t twist_tsc = 0, scan_tsc = 0;  // DPPO_PAR_DBG_CHUNKS: time stamp counts
  // outputs of the stitch
  std::vector<Op> ops;
  std::vector<int32_t> lits;
  int64_t kt0 = 0, kt1 = 0;
};

struct Draw {
  int64_t n = 0, K = 0;
  double inv_n1 = 0;  // 1 / (n - 1)
  int32_t count = 0;
  int P0 = 0;
  const uint32_t* key0 = nullptr;
  std::vector<int64_t> bounds;  // band changes (sorted), the draw's end K included
  // overlap of the phases (par_draw): chunk c's scan done / its stitch done (null: sequential)
  std::atomic<int>* scanned = nullptr;
  std::atomic<int>* stitched = nullptr;
  void wait_scanned(size_t c) const {
    if (!scanned) return;
    for (int k = 0; !scanned[c].load(std::memory_order_acquire); ++k)
      if (k > 64) std::this_thread::yield();
      else _mm_pause();
  }
  void mark_stitched(size_t c0, size_t c1) const {  // chunks [c0, c1)
    if (!stitched) return;
    for (size_t c = c0; c < c1; ++c) stitched[c].store(1, std::memory_order_release);
  }
  Model model;
  std::vector<Chunk> ch;

  int band(int64_t k) const {  // band id of counter k (-1: the draw is done)
    if (k >= K) return -1;
    // the epoch k / (n - 1) by a double reciprocal, corrected by one step either way (the
    // stitch calls this per replayed word; a 64-bit division was its largest single cost)
    int64_t e = (int64_t)((double)k * inv_n1);
    if (e * (n - 1) > k) --e;
    else if ((e + 1) * (n - 1) <= k) ++e;
    const uint32_t i = (uint32_t)(n - 1 - (k - e * (n - 1)));
    return (int)(e * 64 + (31 - __builtin_clz(i)));
  }
  int64_t next_bound(int64_t k) const {  // smallest band change > k
    auto it = std::upper_bound(bounds.begin(), bounds.end(), k);
    return it == bounds.end() ? INT64_MAX : *it;
  }
};

// scan state of one run: counter k, index i, mask, band floor lo
struct Run {
  int64_t k, e;  // counter, epoch
  uint32_t i, mask, lo;
  bool done;
};
// same band: same epoch and band floor (or both done)
inline bool same_band(const Run& a, const Run& b) {
  return a.done ? b.done : (!b.done && a.e == b.e && a.lo == b.lo);
}
inline void run_set(const Draw& D, Run& r, int64_t k) {
  r.k = k;
  r.e = 0;
  r.done = k >= D.K;
  if (r.done) {
    r.i = 0;
    r.mask = 0;
    r.lo = 0;
    return;
  }
  const int64_t e = k / (D.n - 1);
  r.e = e;
  r.i = (uint32_t)(D.n - 1 - (k - e * (D.n - 1)));
  r.mask = smear(r.i);
  r.lo = (r.mask >> 1) + 1;
}
inline void run_accept(const Draw& D, Run& r) {  // after an accept
  ++r.k;
  if (r.done) return;
  if (--r.i >= r.lo) return;
  if (r.k >= D.K) {
    r.done = true;
    r.i = r.mask = r.lo = 0;
    return;
  }
  if (r.i == 0) {  // next epoch
    r.i = (uint32_t)(D.n - 1);
    ++r.e;
  }
  r.mask = smear(r.i);
  r.lo = (r.mask >> 1) + 1;
}

// One chunk's guessed run: targets into C.S, near misses into C.rec, the kept zones.  Groups of
// 16 words take one AVX-512 step where nothing in them can change the band or the zone state and
// no word is ambiguous (perm.cpp's draw_groups_avx512 argument: every v <= i - 15 is accepted and
// every v > i rejected whatever the others do); everything else goes word by word.
PAR_AVX512 void scan_chunk(const Draw& D, Chunk& C, bool last, int64_t est_targets) {
  const auto t0 = std::chrono::steady_clock::now();
  alignas(64) uint32_t mt[kN];
  alignas(64) uint32_t out[kN + 16];
  int64_t blk = C.block0;
  int opos = C.off0;
  if (C.block0 == 0) {
    std::memcpy(mt, D.key0, sizeof(uint32_t) * kN);
    for (int j = opos; j < kN; ++j) out[j] = temper1(mt[j]);
  } else {
    key_after_blocks(D.key0, C.block0, mt);
    for (int j = 0; j < kN; ++j) out[j] = temper1(mt[j]);
  }
  C.jump_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  int64_t scalar_words = 0;
  const int64_t key_from = D.K - C.Wb - 2 * kN;  // keep block keys from this guessed counter on
  Run r;
  run_set(D, r, C.kg0);
  const int64_t stop_k = D.K + C.Wb + 2 * kN;  // the open-ended chunk runs this far past the end
  // zones: the guessed counter within Wb of a band change; `toggle` = counter of the next change
  size_t zi = 0;
  bool zone = false;
  int64_t toggle = INT64_MAX;
  auto zone_state = [&](int64_t k) {
    while (zi < C.zone_iv.size() && C.zone_iv[zi].second < k) ++zi;
    if (zi >= C.zone_iv.size()) {
      zone = false;
      toggle = INT64_MAX;
    } else if (C.zone_iv[zi].first <= k) {
      zone = true;
      toggle = C.zone_iv[zi].second + 1;
    } else {
      zone = false;
      toggle = C.zone_iv[zi].first;
    }
  };
  zone_state(r.k);
  // buffers (kept across calls: sized once)
  const int64_t cap = est_targets + 4 * C.W + 65536;
  if ((int64_t)C.S.size() < cap) C.S.resize((size_t)cap);
  C.rq.clear();
  C.rs.clear();
  C.rm.clear();
  C.ru.clear();
  auto record = [&](uint32_t rq, int64_t rs, int64_t u, uint32_t m) {
    C.rq.push_back(rq);
    C.rs.push_back((uint32_t)rs);
    C.ru.push_back((int32_t)u);
    C.rm.push_back(m);
  };
  C.zones.clear();
  C.key_blocks.clear();
  C.keys.clear();
  C.nraw = 0;
  if (C.raw.size() < 4096) C.raw.resize(4096);
  if (C.bits.size() < 4096 / 64 + 4) C.bits.resize(4096 / 64 + 4);
  std::fill(C.bits.begin(), C.bits.end(), 0);
  auto raw_room = [&](int64_t need) {
    if (C.nraw + need <= (int64_t)C.raw.size()) return;
    const size_t nr = (size_t)((C.nraw + need) * 3 / 2 + 4096);
    C.raw.resize(nr);
    C.bits.resize(nr / 64 + 4, 0);
  };
  auto keep = [&](uint32_t w, bool acc) {
    raw_room(1);
    C.raw[(size_t)C.nraw] = w;
    if (acc) C.bits[(size_t)(C.nraw >> 6)] |= 1ull << (C.nraw & 63);
    ++C.nraw;
  };
  if (zone) C.zones.push_back(Zone{0, 0, C.nraw, r.k});
  if (r.k >= key_from) {
    C.key_blocks.push_back(blk);
    C.keys.insert(C.keys.end(), mt, mt + kN);
  }
  const int64_t W = C.W;  // < 0: no near misses (chunk 0 starts exact)
  int32_t* S = C.S.data();
  int64_t ns = 0;  // guessed targets stored
  int64_t scap = (int64_t)C.S.size() - 32;
  uint32_t q = 0;
  static const bool dbg_tsc = std::getenv("DPPO_PAR_DBG_CHUNKS") != nullptr;
  C.twist_tsc = 0;
  const uint64_t ts0 = dbg_tsc ? __rdtsc() : 0;
  for (;;) {
    if (!last && (int64_t)q >= C.len) break;
    if (last && r.k >= stop_k) break;
    if (opos == kN) {
      const uint64_t tt0 = dbg_tsc ? __rdtsc() : 0;
      twist_temper(mt, out);
      if (dbg_tsc) C.twist_tsc += __rdtsc() - tt0;
      ++blk;
      opos = 0;
      if (r.k >= key_from) {
        C.key_blocks.push_back(blk);
        C.keys.insert(C.keys.end(), mt, mt + kN);
      }
    }
    if (ns + 64 > scap) {
      C.S.resize(C.S.size() * 3 / 2 + 65536);
      S = C.S.data();
      scap = (int64_t)C.S.size() - 32;
    }
    // ---- 64 words at once: one threshold pair for the whole group (every v <= i - 63 is
    // accepted and every v > i rejected whatever the others do), so the loop-carried chain
    // (threshold -> compare -> popcount -> i) runs once per 64 words instead of per 16; a group
    // with a word in (i - 63, i] falls through to the 16-word step
    if (!r.done && opos + 64 <= kN && (last || (int64_t)q + 64 <= C.len) &&
        r.i >= r.lo + 63 && r.k + 64 < toggle && r.k + 64 < D.K) {
      const uint32_t ii = r.i;
      const __m512i vm = _mm512_set1_epi32((int)r.mask);
      const __m512i ta = _mm512_set1_epi32((int)(ii - 63));
      const __m512i tl = _mm512_set1_epi32((int)ii);
      __m512i v[4];
      __mmask16 a16[4];
      uint64_t acc = 0, le = 0;
      for (int g = 0; g < 4; ++g) {
        v[g] = _mm512_and_si512(_mm512_loadu_si512((const void*)(out + opos + 16 * g)), vm);
        a16[g] = _mm512_cmple_epu32_mask(v[g], ta);
        acc |= (uint64_t)a16[g] << (16 * g);
        le |= (uint64_t)_mm512_cmple_epu32_mask(v[g], tl) << (16 * g);
      }
      if (!(le & ~acc)) {
        if (W >= 0) {
          // near misses: u = v - i_l in [-W + 1, W] needs v in (ii - 63 - W, ii + W]
          const __m512i nlo = _mm512_set1_epi32((int)std::max<int64_t>((int64_t)ii - 63 - W, -1));
          const __m512i nhi = _mm512_set1_epi32((int)std::min<int64_t>((int64_t)ii + W, 0x7FFFFFFF));
          uint64_t near = 0;
          for (int g = 0; g < 4; ++g)
            near |= (uint64_t)(_mm512_cmpgt_epi32_mask(v[g], nlo) &
                               _mm512_cmple_epi32_mask(v[g], nhi)) << (16 * g);
          if (near) {
            alignas(64) uint32_t vl[64];
            for (int g = 0; g < 4; ++g) _mm512_store_si512((void*)(vl + 16 * g), v[g]);
            const int64_t s0 = r.k - C.kg0;
            for (uint64_t nm = near; nm; nm &= nm - 1) {
              const int l = __builtin_ctzll(nm);
              const int before = __builtin_popcountll(acc & ((1ull << l) - 1));
              const int64_t u = (int64_t)vl[l] - ((int64_t)ii - before);
              if (u <= W && u >= -W) record(q + (uint32_t)l, s0 + before, u, vl[l]);
            }
          }
        }
        for (int g = 0; g < 4; ++g) {
          _mm512_storeu_si512((void*)(S + ns), _mm512_maskz_compress_epi32(a16[g], v[g]));
          ns += __builtin_popcount((unsigned)a16[g]);
        }
        if (zone) {
          raw_room(64);
          for (int g = 0; g < 4; ++g)
            _mm512_storeu_si512((void*)(C.raw.data() + C.nraw + 16 * g),
                                _mm512_loadu_si512((const void*)(out + opos + 16 * g)));
          const int sh = (int)(C.nraw & 63);
          C.bits[(size_t)(C.nraw >> 6)] |= acc << sh;
          if (sh) C.bits[(size_t)(C.nraw >> 6) + 1] |= acc >> (64 - sh);
          C.nraw += 64;
        }
        const int cnt = __builtin_popcountll(acc);
        q += 64;
        opos += 64;
        r.k += cnt;
        r.i -= (uint32_t)cnt;
        if (r.i < r.lo) {  // one band down (i >= lo - 1 >= 1 here)
          r.mask = smear(r.i);
          r.lo = (r.mask >> 1) + 1;
        }
        continue;
      }
    }
    // ---- 16 words at once
    if (!r.done && opos + 16 <= kN && (last || (int64_t)q + 16 <= C.len) &&
        r.i >= r.lo + 15 && r.k + 16 < toggle && r.k + 16 < D.K) {
      const uint32_t ii = r.i;
      const __m512i v = _mm512_and_si512(_mm512_loadu_si512((const void*)(out + opos)),
                                         _mm512_set1_epi32((int)r.mask));
      const __mmask16 acc = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)(ii - 15)));
      const __mmask16 le = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)ii));
      if (!(le & ~acc)) {
        const int64_t lo_n = (int64_t)ii - 15 - W;
        const int64_t hi_n = (int64_t)ii + W;
        const __mmask16 near =
            _mm512_cmpgt_epi32_mask(v, _mm512_set1_epi32((int)std::max<int64_t>(lo_n, -1))) &
            _mm512_cmple_epi32_mask(v, _mm512_set1_epi32((int)std::min<int64_t>(hi_n, 0x7FFFFFFF)));
        const uint32_t a = (uint32_t)acc;
        const int cnt = __builtin_popcount(a);
        if (near && W >= 0) {
          alignas(64) uint32_t vl[16];
          _mm512_store_si512((void*)vl, v);
          const int64_t s0 = r.k - C.kg0;
          for (uint32_t nm = (uint32_t)near; nm; nm &= nm - 1) {
            const int l = __builtin_ctz(nm);
            const int before = __builtin_popcount(a & ((1u << l) - 1));
            const int64_t u = (int64_t)vl[l] - ((int64_t)ii - before);
            if (u <= W && u >= -W)
              record(q + (uint32_t)l, s0 + before, u, vl[l]);
          }
        }
        _mm512_storeu_si512((void*)(S + ns), _mm512_maskz_compress_epi32(acc, v));
        ns += cnt;
        if (zone) {
          raw_room(16);
          _mm512_storeu_si512((void*)(C.raw.data() + C.nraw),
                              _mm512_loadu_si512((const void*)(out + opos)));
          const int sh = (int)(C.nraw & 63);
          C.bits[(size_t)(C.nraw >> 6)] |= (uint64_t)a << sh;
          if (sh > 48) C.bits[(size_t)(C.nraw >> 6) + 1] |= (uint64_t)a >> (64 - sh);
          C.nraw += 16;
        }
        q += 16;
        opos += 16;
        r.k += cnt;
        r.i -= (uint32_t)cnt;
        if (r.i < r.lo) {  // one band down (i >= lo - 1 >= 1 here)
          r.mask = smear(r.i);
          r.lo = (r.mask >> 1) + 1;
        }
        continue;
      }
    }
    // ---- one word
    ++scalar_words;
    const uint32_t w = out[opos++];
    if (!r.done) {
      const uint32_t v = w & r.mask;
      const bool acc = v <= r.i;
      const int64_t u = (int64_t)v - (int64_t)r.i;
      if (u <= W && u >= -W) record(q, r.k - C.kg0, u, v);
      if (zone) keep(w, acc);
      if (acc) {
        S[ns++] = (int32_t)v;
        run_accept(D, r);
        if (r.k == D.K) C.q_done = q + 1;
      }
    } else {  // past the end: every word counts (the stitcher only needs the words)
      if (zone) keep(w, true);
      ++r.k;
    }
    ++q;
    if (r.k >= toggle) {
      if (zone) C.zones.back().q1 = q;
      zone_state(r.k);
      if (zone) C.zones.push_back(Zone{q, 0, C.nraw, r.k});
    }
    if (q >= 0xFFFFFF00u) {
      C.overflow = true;
      break;
    }
  }
  if (zone) C.zones.back().q1 = q;
  if (dbg_tsc) C.scan_tsc = __rdtsc() - ts0;
  C.words = q;
  C.scalar_words = scalar_words;
  C.kg_end = r.k;
  C.ns = ns;
  // accept-count prefix of the kept words, per 64
  const size_t nb = (size_t)(C.nraw >> 6) + 2;
  C.pref.resize(nb + 1);
  uint32_t acc_sum = 0;
  for (size_t b = 0; b <= nb; ++b) {
    C.pref[b] = acc_sum;
    if (b < nb) acc_sum += (uint32_t)__builtin_popcountll(C.bits[b]);
  }
  C.us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

// ------------------------------------------------------------------------------------------
// The stitch: the true run through every chunk, as copies of guessed targets plus literals
// ------------------------------------------------------------------------------------------
struct Stitch {
  const Draw& D;
  explicit Stitch(const Draw& d) : D(d) {}
  int64_t exact_words = 0, max_delta = 0, triggers = 0;
  double wait_us = 0;     // time spent waiting for chunk scans (stats: the stitch's own work)
  int fail = 0;           // reason code of a failed stitch
  int64_t end_word = -1;  // global index of the word after the last accepted one

  Chunk* C = nullptr;
  int64_t kt = 0;          // true counter
  int64_t s = 0;           // guessed targets passed (guessed counter kg = kg0 + s)
  int64_t cs = 0, ck = 0;  // pending copy: guessed index cs -> true counter ck
  size_t ri = 0;           // next record
  Run tr{};                // the true run (EXACT)

  int64_t kg() const { return C->kg0 + s; }
  int64_t d() const { return kg() - kt; }
  void flush() {
    if (s > cs) C->ops.push_back(Op{ck, cs, s - cs, 0});
    cs = s;
    ck = kt;
  }
  void literal(uint32_t v) {
    if (!C->ops.empty() && C->ops.back().lit && C->ops.back().k + C->ops.back().len == kt &&
        C->ops.back().src + C->ops.back().len == (int64_t)C->lits.size()) {
      C->ops.back().len++;
    } else {
      C->ops.push_back(Op{kt, (int64_t)C->lits.size(), 1, 1});
    }
    C->lits.push_back((int32_t)v);
    ++kt;
  }
  // up to 16 literals at once: the accepted lanes of v, in lane order
  PAR_AVX512 void literals(__m512i v, __mmask16 acc, int cnt) {
    if (!cnt) return;
    const size_t base = C->lits.size();
    C->lits.resize(base + 16);
    _mm512_storeu_si512((void*)(C->lits.data() + base), _mm512_maskz_compress_epi32(acc, v));
    C->lits.resize(base + (size_t)cnt);
    if (!C->ops.empty() && C->ops.back().lit && C->ops.back().k + C->ops.back().len == kt &&
        C->ops.back().src + C->ops.back().len == (int64_t)base)
      C->ops.back().len += cnt;
    else
      C->ops.push_back(Op{kt, (int64_t)base, cnt, 1});
    kt += cnt;
  }
  // no disagreement up to guessed index s2: the copy extends
  void advance_to(int64_t s2) {
    kt += s2 - s;
    s = s2;
  }
  bool check_d() {
    const int64_t x = d();
    max_delta = std::max(max_delta, x < 0 ? -x : x);
    const int64_t w = std::max<int64_t>(C->W, 0);
    if (x > w || x < -w) {
      fail = 2;
      return false;
    }
    return true;
  }
  // The first record at or after ri with word < qlim on which the two runs disagree under the
  // current offset (d > 0: masked value in (i_g, i_g + d]; d < 0: in (i_g + d, i_g]); else the
  // first record with word >= qlim.
  PAR_AVX512 size_t next_trigger(int64_t qlim) const {
    const size_t end = C->rq.size();
    const int64_t dd = d();
    const int32_t lo = (int32_t)(dd > 0 ? 0 : dd), hi = (int32_t)(dd > 0 ? dd : 0);
    const uint32_t ql = (uint32_t)std::min<int64_t>(qlim, 0xFFFFFFFFll);
    const int32_t* u = C->ru.data();
    const uint32_t* rq = C->rq.data();
    size_t j = ri;
    const __m512i vlo = _mm512_set1_epi32(lo), vhi = _mm512_set1_epi32(hi),
                  vq = _mm512_set1_epi32((int)ql);
    for (; j + 16 <= end; j += 16) {
      const __m512i x = _mm512_loadu_si512((const void*)(u + j));
      const __m512i y = _mm512_loadu_si512((const void*)(rq + j));
      const __mmask16 m = (_mm512_cmpgt_epi32_mask(x, vlo) & _mm512_cmple_epi32_mask(x, vhi)) |
                          _mm512_cmpge_epu32_mask(y, vq);
      if (m) return j + (size_t)__builtin_ctz((unsigned)m);
    }
    for (; j < end; ++j)
      if ((u[j] > lo && u[j] <= hi) || rq[j] >= ql) return j;
    return end;
  }
  // apply disagreeing record j; the word after it becomes the current word
  bool take(size_t j) {
    ++triggers;
    advance_to(C->rs[j]);
    flush();
    if (C->ru[j] > 0) {  // only the true run accepts (d > 0)
      literal(C->rm[j]);
    } else {             // only the guessed run accepts (d < 0)
      ++s;
    }
    cs = s;
    ck = kt;
    ri = j + 1;
    return check_d();
  }
  // accepts among kept words [0, x) of the chunk
  int64_t P(int64_t x) const {
    const int64_t b = x >> 6;
    const int r = (int)(x & 63);
    return C->pref[(size_t)b] +
           (r ? __builtin_popcountll(C->bits[(size_t)b] & ((1ull << r) - 1)) : 0);
  }
  int64_t zone_count(const Zone& z, int64_t qa, int64_t qb) const {  // accepts in [qa, qb)
    return P(z.raw0 + (qb - z.q0)) - P(z.raw0 + (qa - z.q0));
  }
  // the word just after the guessed counter reaches `target`, from word q of zone z where it
  // is kg; -1 if not inside the zone
  PAR_AVX512 int64_t zone_reach(const Zone& z, int64_t q, int64_t kgq, int64_t target) const {
    if (kgq >= target) return q;
    const int64_t xa = z.raw0 + (q - z.q0);
    const int64_t xe = z.raw0 + (z.q1 - z.q0);
    const int64_t need = P(xa) + (target - kgq);  // the first x with P(x + 1) >= need
    if (P(xe) < need) return -1;
    int64_t lo = xa >> 6, hi = (xe >> 6) + 1;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if ((int64_t)C->pref[(size_t)mid] >= need) hi = mid;
      else lo = mid;
    }
    const uint64_t word = C->bits[(size_t)lo];
    const int64_t j = need - C->pref[(size_t)lo];  // >= 1
    const uint64_t sel = _pdep_u64(1ull << (j - 1), word);
    const int64_t x = lo * 64 + __builtin_ctzll(sel);
    return z.q0 + (x - z.raw0) + 1;
  }
};

// Runs the stitch over all chunks; fills ops / lits; returns false on any failed check.
PAR_AVX512 bool stitch_all(Draw& D, Stitch& X) {
  enum { OFFSET, EXACT, LOCKED } mode = OFFSET;
  int64_t kt = 0;
  for (size_t c = 0; c < D.ch.size(); ++c) {
    {
      const auto w0 = std::chrono::steady_clock::now();
      D.wait_scanned(c);
      X.wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0)
                       .count();
    }
    if (c > 0) D.mark_stitched(c - 1, c);  // chunk c-1's ops are final
    Chunk& C = D.ch[c];
    // every disagreement is a record (~1/6 of them disagree in practice) and costs at most two
    // ops and a literal; the replayed zone words add literals: reserved up front from those
    // counts, so the vectors rarely grow inside the serial stitch (growing them there cost ~3x
    // per trigger in the draws that outgrew the previous capacity)
    {
      const size_t nops = C.rq.size() + (size_t)C.zones.size() * 64 + 1024;
      const size_t nlits = C.rq.size() + (size_t)C.nraw + 1024;
      if (C.ops.capacity() < nops) C.ops.reserve(nops);
      if (C.lits.capacity() < nlits) C.lits.reserve(nlits);
    }
    X.C = &C;
    X.kt = kt;
    X.s = 0;
    X.cs = 0;
    X.ck = kt;
    X.ri = 0;
    C.kt0 = kt;
    if (C.overflow) {
      X.fail = 9;
      return false;
    }
    int64_t q = 0;
    size_t zi = 0;
    if (mode == EXACT || D.band(C.kg0) != D.band(kt)) {
      mode = EXACT;
    } else {
      if (!X.check_d()) {
        X.fail = 1;
        return false;
      }
      mode = X.d() == 0 ? LOCKED : OFFSET;
    }
    const int64_t words = C.words;
    for (;;) {
      if (mode == LOCKED) {  // the true run IS the guessed run from word q on
        if (C.q_done >= 0) {
          if (C.q_done < q) {
            X.fail = 8;
            return false;
          }
          X.advance_to(D.K - C.kg0);
          X.flush();
          X.end_word = C.Q0 + C.q_done;
          C.kt1 = X.kt;
          D.mark_stitched(c, D.ch.size());
          return true;
        }
        X.advance_to(C.kg_end - C.kg0);
        break;
      }
      if (mode == OFFSET) {
        while (zi < C.zones.size() && C.zones[zi].q1 <= q) ++zi;
        const bool inz = zi < C.zones.size() && C.zones[zi].q0 <= q;
        if (!inz) {  // same band until the next zone: only disagreeing records matter
          const int64_t qz = zi < C.zones.size() ? C.zones[zi].q0 : words;
          // neither run may change band before the next zone (the zones are built so that it
          // cannot; checked, not assumed)
          const int64_t guard_t = D.next_bound(X.kt), guard_g = D.next_bound(X.kg());
          if (D.band(X.kt) != D.band(X.kg())) {
            X.fail = 11;
            return false;
          }
          bool locked = false;
          for (;;) {
            const size_t j = X.next_trigger(qz);
            if (j >= C.rq.size() || C.rq[j] >= qz) {
              X.ri = j;
              break;
            }
            if (!X.take(j)) return false;
            q = C.rq[j] + 1;
            if (X.kt >= guard_t || X.kg() >= guard_g) {
              X.fail = 12;
              return false;
            }
            if (X.d() == 0) {
              locked = true;
              break;
            }
          }
          if (locked) {
            mode = LOCKED;
            continue;
          }
          if (zi >= C.zones.size()) {
            X.advance_to(C.kg_end - C.kg0);
            if (X.kt >= guard_t || X.kg() >= guard_g) {
              X.fail = 12;
              return false;
            }
            break;
          }
          X.advance_to(C.zones[zi].k0 - C.kg0);
          // arriving exactly on a band change (counter == guard) is allowed: the zone handles it
          if (X.kt > guard_t || X.kg() > guard_g) {
            X.fail = 12;
            return false;
          }
          q = C.zones[zi].q0;
          continue;
        }
        if (D.band(X.kt) != D.band(X.kg())) {  // entering or inside a zone in different bands
          mode = EXACT;
          continue;
        }
        // inside zone zi, both runs in one band: where does the leader change band?
        const Zone& z = C.zones[zi];
        const int64_t Kb = D.next_bound(std::max(X.kg(), X.kt));
        if (X.d() > 0) {  // the guessed run leads and changes band first, at word qg
          const int64_t qg = X.zone_reach(z, q, X.kg(), Kb);
          const int64_t qlim = qg < 0 ? (int64_t)z.q1 : qg;
          bool locked = false;
          for (;;) {
            const size_t j = X.next_trigger(qlim);
            if (j >= C.rq.size() || C.rq[j] >= qlim) {
              X.ri = j;
              break;
            }
            if (!X.take(j)) return false;
            q = C.rq[j] + 1;
            if (X.d() == 0) {
              locked = true;
              break;
            }
          }
          if (locked) {
            mode = LOCKED;
            continue;
          }
          if (qg < 0) {
            X.advance_to(z.k0 + X.zone_count(z, z.q0, z.q1) - C.kg0);
            q = z.q1;
            ++zi;
            continue;
          }
          X.advance_to(Kb - C.kg0);
          q = qg;
          mode = EXACT;
          continue;
        }
        // the true run leads: it changes band when the guessed counter reaches Kb + d
        bool locked = false, found = false;
        for (;;) {
          const int64_t kap = Kb + X.d();
          const int64_t qs = X.zone_reach(z, q, X.kg(), kap);
          const int64_t qlim = qs < 0 ? (int64_t)z.q1 : qs;
          const size_t j = X.next_trigger(qlim);
          if (j < C.rq.size() && C.rq[j] < qlim) {
            if (!X.take(j)) return false;
            q = C.rq[j] + 1;
            if (X.d() == 0) {
              locked = true;
              break;
            }
            continue;
          }
          X.ri = j;
          if (qs < 0) break;
          X.advance_to(kap - C.kg0);
          q = qs;
          found = true;
          break;
        }
        if (locked) {
          mode = LOCKED;
          continue;
        }
        if (!found) {
          X.advance_to(z.k0 + X.zone_count(z, z.q0, z.q1) - C.kg0);
          q = z.q1;
          ++zi;
          continue;
        }
        mode = EXACT;
        continue;
      }
      // EXACT: the runs are in different bands; replay the true run over the kept words
      while (zi < C.zones.size() && C.zones[zi].q1 <= q) ++zi;
      if (zi >= C.zones.size() || C.zones[zi].q0 > q) {
        X.fail = 3;
        return false;
      }
      const Zone& z = C.zones[zi];
      int64_t kgq = z.k0 + X.zone_count(z, z.q0, q);
      X.s = kgq - C.kg0;
      X.flush();
      run_set(D, X.tr, X.kt);
      const uint32_t* rw = C.raw.data() + z.raw0 - z.q0;
      const int64_t bo = z.raw0 - z.q0;
      bool back = false;
      int64_t x = q;
      while (x < (int64_t)z.q1) {
        // 16 words at once where the true run can neither change band, finish, nor meet an
        // ambiguous word (the scan's group step); the guessed counter advances by the popcount
        // of its 16 accept bits
        if (!X.tr.done && x + 16 <= (int64_t)z.q1 && X.tr.i >= X.tr.lo + 15 &&
            X.tr.k + 16 < D.K) {
          const uint32_t ii = X.tr.i;
          const __m512i v = _mm512_and_si512(_mm512_loadu_si512((const void*)(rw + x)),
                                             _mm512_set1_epi32((int)X.tr.mask));
          const __mmask16 acc = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)(ii - 15)));
          const __mmask16 le = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)ii));
          if (!(le & ~acc)) {
            const int cnt = __builtin_popcount((unsigned)acc);
            X.literals(v, acc, cnt);
            X.tr.k += cnt;
            X.tr.i -= (uint32_t)cnt;
            if (X.tr.i < X.tr.lo) {
              X.tr.mask = smear(X.tr.i);
              X.tr.lo = (X.tr.mask >> 1) + 1;
            }
            const int64_t b = x + bo;
            const int o = (int)(b & 63);
            uint64_t w16 = C.bits[(size_t)(b >> 6)] >> o;
            if (o > 48) w16 |= C.bits[(size_t)(b >> 6) + 1] << (64 - o);
            const int gcnt = __builtin_popcountll(w16 & 0xFFFFull);
            kgq += gcnt;
            x += 16;
            X.exact_words += 16;
            if ((cnt || gcnt) && D.band(kgq) == D.band(X.kt)) {
              back = true;
              break;
            }
            continue;
          }
        }
        ++X.exact_words;
        bool moved = false;
        if (!X.tr.done) {
          const uint32_t v = rw[x] & X.tr.mask;
          if (v <= X.tr.i) {
            X.literal(v);
            run_accept(D, X.tr);
            if (X.tr.k == D.K) {
              X.end_word = C.Q0 + x + 1;
              C.kt1 = X.kt;
              D.mark_stitched(c, D.ch.size());
              return true;
            }
            moved = true;
          }
        }
        if ((C.bits[(size_t)((x + bo) >> 6)] >> ((x + bo) & 63)) & 1) {
          ++kgq;
          moved = true;
        }
        ++x;
        if (moved && D.band(kgq) == D.band(X.kt)) {
          back = true;
          break;
        }
      }
      q = x;
      X.s = kgq - C.kg0;
      X.cs = X.s;
      X.ck = X.kt;
      if (back) {
        X.ri = (size_t)(std::lower_bound(C.rq.begin(), C.rq.end(), (uint32_t)q) - C.rq.begin());
        if (!X.check_d()) {
          X.fail = 4;
          return false;
        }
        mode = X.d() == 0 ? LOCKED : OFFSET;
        continue;
      }
      if (q >= words && c + 1 < D.ch.size()) break;  // still different bands: EXACT goes on
      X.fail = 5;
      return false;
    }
    if (mode != EXACT) X.flush();
    kt = X.kt;
    C.kt1 = kt;
  }
  X.fail = 6;  // ran out of words
  return false;
}

// ------------------------------------------------------------------------------------------
// Assembly and the worker pool
// ------------------------------------------------------------------------------------------
// dst[-j] = src[j], j < len.  The destination (the pinned upload slot) is written with
// non-temporal 64-B stores where aligned: no read-for-ownership of lines that are only written,
// and the CPU caches are left to the scan.
PAR_AVX512 void copy_reversed(int32_t* dst, const int32_t* src, int64_t len) {
  const __m512i rev = _mm512_set_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  int64_t j = 0;
  // head: until dst - j + 1 (the end of the next 16-element block) is 64-B aligned
  while (j < len && (((uintptr_t)(dst - j + 1)) & 63) != 0) {
    dst[-j] = src[j];
    ++j;
  }
  for (; j + 16 <= len; j += 16)
    _mm512_stream_si512((__m512i*)(dst - j - 15),
                        _mm512_permutexvar_epi32(rev, _mm512_loadu_si512((const void*)(src + j))));
  for (; j < len; ++j) dst[-j] = src[j];
}

void assemble_chunk(const Draw& D, const Chunk& C, int32_t* out) {
  const int64_t n1 = D.n - 1;
  for (const Op& op : C.ops) {
    const int32_t* src = (op.lit ? C.lits.data() : C.S.data()) + op.src;
    int64_t k = op.k, left = op.len;
    while (left > 0) {
      const int64_t e = k / n1;
      const int64_t r = k - e * n1;          // position in the epoch; index i = n-1-r
      const int64_t run = std::min(left, n1 - r);
      int32_t* dst = out + e * D.n + (D.n - 1 - r);
      copy_reversed(dst, src, run);
      src += run;
      k += run;
      left -= run;
    }
  }
}

class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool();  // leaked on purpose: no join at process exit
    return *p;
  }
  // helpers (threads - 1 workers) run `body` while the caller does other work; wait() returns
  // once every helper has left it.  One session at a time (the lock).
  class Session {
   public:
    Session(Pool& p, int helpers, std::function<void()> body) : p_(p), lk_(p.run_mu_) {
      p_.ensure(helpers);
      std::lock_guard<std::mutex> g(p_.mu_);
      p_.task_ = std::move(body);
      p_.helpers_ = std::min(helpers, (int)p_.workers_.size());
      p_.gen_++;
      p_.cv_.notify_all();
    }
    void wait() {
      std::unique_lock<std::mutex> g(p_.mu_);
      // a helper that has not picked the task up yet must not start it late: clear it first
      p_.task_ = nullptr;
      p_.done_cv_.wait(g, [&] { return p_.active_ == 0; });
    }
    ~Session() { wait(); }

   private:
    Pool& p_;
    std::lock_guard<std::mutex> lk_;
  };

  // runs fn(0 .. jobs-1) on `threads` threads (the caller is one of them)
  void run(int jobs, int threads, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> serial(run_mu_);
    ensure(threads - 1);
    std::atomic<int> next{0};
    std::atomic<int> left{jobs};
    auto body = [&] {
      for (int j; (j = next.fetch_add(1)) < jobs;) {
        fn(j);
        left.fetch_sub(1);
      }
    };
    {
      std::lock_guard<std::mutex> g(mu_);
      task_ = body;
      helpers_ = std::min(threads - 1, (int)workers_.size());
      gen_++;
    }
    cv_.notify_all();
    body();
    while (left.load() > 0) std::this_thread::yield();
    // every helper must have left `body` before its captures go out of scope
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return active_ == 0; });
    task_ = nullptr;
  }

 private:
  void ensure(int nw) {
    std::lock_guard<std::mutex> g(mu_);
    while ((int)workers_.size() < nw) {
      const int id = (int)workers_.size();
      workers_.emplace_back([this, id] { loop(id); });
      // Helper k runs on a physical core of its own (one logical CPU per core of the affinity
      // mask; DPPO_PERM_PAR_PIN=0 leaves placement to the scheduler).  Left to the scheduler on
      // the box's shared 256-CPU host, helpers landed on busy or sibling CPUs: the MT19937 twist
      // -- pure L1 compute -- ran 0.66 TSC ticks per word at the median instead of 0.36, and a
      // chained draw took 7.0-7.4 ms instead of 5.0-5.4 at 12 threads (tools/gpu/r05_draw_pin.sh).
      const char* e = std::getenv("DPPO_PERM_PAR_PIN");
      if (!(e && e[0] == '0')) {
        const std::vector<int>& cores = pin_cores();
        if (!cores.empty()) {
          // DPPO_PERM_PAR_PIN=2 (A/B): the block taken from the far end of the list
          const size_t k = (pin_base() + id + 1) % cores.size();
          const size_t at = (e && e[0] == '2') ? cores.size() - 1 - k : k;
          cpu_set_t set;
          CPU_ZERO(&set);
          CPU_SET(cores[at], &set);
          pthread_setaffinity_np(workers_.back().native_handle(), sizeof(set), &set);
        }
      }
      workers_.back().detach();
    }
  }
  // Where this process's block of helper cores starts in pin_cores(): with several ranks per
  // node (torchrun's LOCAL_RANK / LOCAL_WORLD_SIZE), rank r takes the cores r x (threads + 1)
  // on, so that the ranks' helpers never share a core; one process starts at the caller's core.
  static size_t pin_base() {
    const char* lr = std::getenv("LOCAL_RANK");
    const char* lw = std::getenv("LOCAL_WORLD_SIZE");
    if (!lr || !lw || std::atoi(lw) <= 1) return 0;
    const char* t = std::getenv("DPPO_PERM_PAR_THREADS");
    const int per = (t ? std::max(1, std::atoi(t)) : 12) + 1;
    return (size_t)std::max(0, std::atoi(lr)) * (size_t)per;
  }
  // one logical CPU per physical core of the affinity mask (in mask order; one process: rotated
  // to start at the caller's core)
  static const std::vector<int>& pin_cores() {
    static const std::vector<int> v = [] {
      std::vector<int> out;
      cpu_set_t m;
      if (sched_getaffinity(0, sizeof(m), &m) != 0) return out;
      std::vector<int> all;
      for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &m)) all.push_back(c);
      std::vector<bool> taken(CPU_SETSIZE, false);
      for (int c : all) {
        if (taken[(size_t)c]) continue;
        out.push_back(c);
        char path[96];
        std::snprintf(path, sizeof(path),
                      "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
        if (FILE* f = std::fopen(path, "r")) {
          int a = -1, b = -1;
          char sep = 0;
          if (std::fscanf(f, "%d%c%d", &a, &sep, &b) >= 1) {
            if (a >= 0 && a < CPU_SETSIZE) taken[(size_t)a] = true;
            if (b >= 0 && b < CPU_SETSIZE) taken[(size_t)b] = true;
          }
          std::fclose(f);
        }
      }
      if (pin_base() == 0) {
        const int me = sched_getcpu();
        auto it = std::find(out.begin(), out.end(), me);
        if (it != out.end()) std::rotate(out.begin(), it, out.end());
      }
      return out;
    }();
    return v;
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= helpers_ || !task_) continue;
        t = task_;
        ++active_;
      }
      t();
      std::lock_guard<std::mutex> g(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void()> task_;
  std::vector<std::thread> workers_;
  uint64_t gen_ = 0;
  int helpers_ = 0, active_ = 0;
};

std::atomic<int64_t> g_par_calls{0}, g_par_ok{0}, g_par_fallback{0};

std::mutex g_chunks_mu;
std::vector<std::unique_ptr<std::vector<Chunk>>> g_chunks_free;
std::unique_ptr<std::vector<Chunk>> take_chunks() {
  std::lock_guard<std::mutex> g(g_chunks_mu);
  if (g_chunks_free.empty()) return std::unique_ptr<std::vector<Chunk>>(new std::vector<Chunk>());
  auto p = std::move(g_chunks_free.back());
  g_chunks_free.pop_back();
  return p;
}
void give_chunks(std::unique_ptr<std::vector<Chunk>>&& p) {
  std::lock_guard<std::mutex> g(g_chunks_mu);
  if (g_chunks_free.size() < 2) g_chunks_free.push_back(std::move(p));
}

bool cpu_ok() {
  static const bool yes = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                          __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq") &&
                          __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("bmi2");
  return yes;
}

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// The parallel draw; false = not done (the caller draws serially).  stats: see dppo.h.
bool par_draw(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out, int threads,
              int64_t chunks, int64_t w_override, double w_mult, int64_t* st) {
  const double t_start = now_us();
  Draw D;
  D.n = n;
  D.inv_n1 = n > 1 ? 1.0 / (double)(n - 1) : 0.0;
  D.count = count;
  D.K = (int64_t)count * (n - 1);
  D.P0 = *pos;
  D.key0 = key;
  D.model.init(n, count);
  if (!field().ok) {
    if (st) st[13] = 10;
    return false;
  }
  // band changes: epoch starts, powers of two inside each epoch, the end
  for (int64_t e = 0; e < count; ++e) {
    const int64_t base = e * (n - 1);
    if (e > 0) D.bounds.push_back(base);
    for (int64_t p = 2; p <= n - 1; p <<= 1) D.bounds.push_back(base + n - p);
  }
  D.bounds.push_back(D.K);
  std::sort(D.bounds.begin(), D.bounds.end());
  D.bounds.erase(std::unique(D.bounds.begin(), D.bounds.end()), D.bounds.end());
  double Etot, Vtot;
  D.model.before(D.K, &Etot, &Vtot);
  // chunks: whole blocks, chunk c >= 1 starting at block c * Lb
  const int64_t C = std::max<int64_t>(1, chunks > 0 ? chunks : 2 * (int64_t)threads);
  // whole blocks per chunk from the model alone (not from pos), so the jump polynomials --
  // x^(624 c Lb - 1) mod phi, ~25 squarings each -- are computed once per configuration
  int64_t Lb = (int64_t)(Etot / (kN * (double)C));
  if (Lb > 64) Lb &= ~(int64_t)15;
  if (Lb < 1 || C < 2) {
    if (st) st[13] = 11;
    return false;
  }
  // chunk buffers are reused across calls (a fresh 134 MB of targets per call costs ~33 K
  // first-touch page faults)
  std::unique_ptr<std::vector<Chunk>> held = take_chunks();
  D.ch.swap(*held);
  struct Give {
    Draw& d;
    std::unique_ptr<std::vector<Chunk>>& h;
    ~Give() {
      d.ch.swap(*h);
      give_chunks(std::move(h));
    }
  } give{D, held};
  D.ch.resize((size_t)C);
  for (Chunk& ch : D.ch) {
    ch.q_done = -1;
    ch.overflow = false;
    ch.ops.clear();
    ch.lits.clear();
  }
  for (int64_t c = 0; c < C; ++c) {
    Chunk& ch = D.ch[(size_t)c];
    if (c == 0) {
      ch.block0 = 0;
      ch.off0 = D.P0;
      ch.Q0 = 0;
      ch.kg0 = 0;
    } else {
      ch.block0 = c * Lb;
      ch.off0 = 0;
      ch.Q0 = kN * ch.block0 - D.P0;
      ch.kg0 = D.model.counter_at((double)ch.Q0);
    }
  }
  for (int64_t c = 0; c + 1 < C; ++c) D.ch[(size_t)c].len = D.ch[(size_t)c + 1].Q0 - D.ch[(size_t)c].Q0;
  D.ch.back().len = -1;
  // per chunk: the near-miss band W = w_mult sigma (the model's word-count deviation at the
  // chunk's first word: how far the true counter may sit from the guess) and the zones; chunk 0
  // starts exact, so its guessed run is the true run (no near misses, no zones)
  int64_t Wmax = 0, Wbmax = 0;
  for (int64_t c = 0; c < C; ++c) {
    Chunk& ch = D.ch[(size_t)c];
    ch.zone_iv.clear();
    if (c == 0) {
      ch.W = -1;
      ch.Wb = 0;
      ch.zone_iv.push_back({D.K - 2 * kN, D.K + 2 * kN});  // the end keys / end words
      continue;
    }
    double E0, V0;
    D.model.before(ch.kg0, &E0, &V0);
    ch.W = w_override > 0 ? w_override : (int64_t)std::ceil(w_mult * std::sqrt(V0)) + 256;
    ch.Wb = 2 * ch.W + 1024;
    for (int64_t b : D.bounds) {
      const int64_t lo = b - ch.Wb, hi = b + ch.Wb;
      if (!ch.zone_iv.empty() && lo <= ch.zone_iv.back().second + 1)
        ch.zone_iv.back().second = std::max(ch.zone_iv.back().second, hi);
      else
        ch.zone_iv.push_back({lo, hi});
    }
    if (std::getenv("DPPO_PAR_DBG_NOREC")) ch.W = -1;
    if (std::getenv("DPPO_PAR_DBG_NOZONE")) ch.zone_iv.clear();
    Wmax = std::max(Wmax, ch.W);
    Wbmax = std::max(Wbmax, ch.Wb);
  }
  // The three phases overlap: the helpers scan chunks in order (then assemble), the caller
  // stitches chunk c as soon as its scan is done, and a chunk is assembled as soon as its stitch
  // is done.  With two chunks per thread the stitch of the first half runs under the scans of the
  // second.
  const double t1 = now_us();
  field();  // build phi before the workers race for it
  const int64_t est = D.K / C + 1;
  std::unique_ptr<std::atomic<int>[]> scanned(new std::atomic<int>[(size_t)C]);
  std::unique_ptr<std::atomic<int>[]> stitched(new std::atomic<int>[(size_t)C]);
  for (int64_t c = 0; c < C; ++c) {
    scanned[c].store(0);
    stitched[c].store(0);
  }
  D.scanned = scanned.get();
  D.stitched = stitched.get();
  // Scan order: the chunks holding an epoch's end (and the last one, the draw's end) first.  There
  // the low mask bands make nearly every word a near miss and keep it in a zone (~170 K records
  // and ~600 K kept words in such a chunk at configs[4], ~8 TSC ticks per word against ~1.7),
  // so one of them took 4-5 ms against ~1.2 ms for the others; scanned last in index order, the
  // last chunk alone set the draw's time.  The stitch still walks the chunks in index order.
  std::vector<int> order;
  {
    std::vector<char> heavy((size_t)C, 0);
    heavy[(size_t)C - 1] = 1;
    for (int64_t e = 1; e < count; ++e) {
      const int64_t kb = e * (n - 1);  // the counter where epoch e starts
      for (int64_t c = 0; c + 1 < C; ++c)
        if (D.ch[(size_t)c].kg0 < kb && kb <= D.ch[(size_t)c + 1].kg0) heavy[(size_t)c] = 1;
    }
    for (int64_t c = 0; c < C; ++c)
      if (heavy[(size_t)c]) order.push_back((int)c);
    for (int64_t c = 0; c < C; ++c)
      if (!heavy[(size_t)c]) order.push_back((int)c);
  }
  std::atomic<int> next_scan{0}, next_asm{0}, abort_asm{0};
  std::atomic<double> scans_done_at{0.0};
  auto assemble_jobs = [&] {
    for (int a; (a = next_asm.fetch_add(1)) < (int)C;) {
      for (int k = 0; !stitched[a].load(std::memory_order_acquire); ++k) {
        if (abort_asm.load(std::memory_order_relaxed)) return;
        if (k > 64) std::this_thread::yield();
        else _mm_pause();
      }
      if (abort_asm.load(std::memory_order_relaxed)) return;
      const Chunk& ch = D.ch[(size_t)a];
      if (!ch.ops.empty()) assemble_chunk(D, ch, out);
      _mm_sfence();  // the non-temporal stores drained before the caller reads or uploads out
    }
  };
  Stitch X(D);
  bool ok = false;
  double t3 = 0;
  {
    Pool::Session ses(Pool::get(), threads - 1, [&] {
      for (int x; (x = next_scan.fetch_add(1)) < (int)C;) {
        const int c = order[(size_t)x];
        scan_chunk(D, D.ch[(size_t)c], c == C - 1, c == C - 1 ? est + est / 4 : est);
        scanned[c].store(1, std::memory_order_release);
        double prev = scans_done_at.load(), t = now_us();
        while (t > prev && !scans_done_at.compare_exchange_weak(prev, t)) {
        }
      }
      assemble_jobs();
    });
    ok = stitch_all(D, X);
    t3 = now_us();
    if (ok) D.mark_stitched(0, (size_t)C);
    else abort_asm.store(1);
    // the caller helps with the last assemblies, then every helper has left the body
    if (ok) assemble_jobs();
    ses.wait();
  }
  const double t2 = scans_done_at.load() > 0 ? scans_done_at.load() : t3;
  int64_t recs = 0, zw = 0, gen = 0;
  double scan_max = 0, jump_max = 0;
  int64_t scal = 0;
  for (const Chunk& ch : D.ch) {
    jump_max = std::max(jump_max, ch.jump_us);
    scal += ch.scalar_words;
    recs += (int64_t)ch.rq.size();
    zw += ch.nraw;
    gen += ch.words;
    scan_max = std::max(scan_max, ch.us);
  }
  if (std::getenv("DPPO_PAR_DBG_CHUNKS"))
    for (const Chunk& ch : D.ch)
      std::fprintf(stderr,
                   "chunk words %lld us %.0f jump %.0f recs %zu raw %lld scalar %lld W %lld "
                   "tsc/word: loop %.2f twist %.2f\n",
                   (long long)ch.words, ch.us, ch.jump_us, ch.rq.size(), (long long)ch.nraw,
                   (long long)ch.scalar_words, (long long)ch.W,
                   (double)ch.scan_tsc / (double)std::max<int64_t>(ch.words, 1),
                   (double)ch.twist_tsc / (double)std::max<int64_t>(ch.words, 1));
  if (st) {
    st[1] = C;
    st[2] = recs;
    st[3] = zw;
    st[4] = X.exact_words;
    st[5] = X.max_delta;
    st[6] = Wmax;
    st[7] = Wbmax;
    st[8] = (int64_t)(t2 - t1);  // the last scan done
    st[9] = (int64_t)(t3 - t1);  // the stitch done (it overlaps the scans)
    st[11] = (int64_t)scan_max;
    st[12] = gen;
    st[13] = ok ? 0 : X.fail;
    st[15] = (int64_t)jump_max;
    st[16] = scal;
    st[17] = X.triggers;
    st[18] = (int64_t)(t3 - t1 - X.wait_us);  // the stitch's own work (its waits excluded)
  }
  if (!ok) return false;
  // the generator state after the last consumed word
  const int64_t last = X.end_word - 1 + D.P0;  // absolute word index (block 0 = key0)
  const int64_t blk = last / kN;
  const int32_t npos = (int32_t)(last % kN) + 1;
  const uint32_t* nkey = nullptr;
  if (blk == 0) {
    nkey = key;
  } else {
    for (const Chunk& ch : D.ch)
      for (size_t j = 0; j < ch.key_blocks.size(); ++j)
        if (ch.key_blocks[j] == blk) nkey = ch.keys.data() + j * kN;
  }
  if (!nkey) {
    if (st) st[13] = 7;
    return false;
  }
  for (int64_t e = 0; e < count; ++e) out[e * n] = 0;
  const double t4 = now_us();
  if (nkey != key) std::memcpy(key, nkey, kN * sizeof(uint32_t));
  *pos = npos;
  if (st) {
    st[10] = (int64_t)(t4 - t3);  // assembly after the stitch
    st[14] = (int64_t)(t4 - t_start);
  }
  return true;
}

}  // namespace

namespace dppo {
// The default path of dppo_perm_targets_numpy for large draws (perm.cpp); true = done.
bool perm_targets_parallel(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out) {
  static const int threads = [] {
    const char* e = std::getenv("DPPO_PERM_PAR_THREADS");
    return e ? std::atoi(e) : 12;
  }();
  static const int64_t min_targets = [] {
    const char* e = std::getenv("DPPO_PERM_PAR_MIN");
    return e ? std::atoll(e) : (int64_t)1 << 22;
  }();
  if (threads < 2 || !cpu_ok() || (int64_t)count * (n - 1) < min_targets) return false;
  g_par_calls.fetch_add(1);
  int64_t st[24] = {0};
  if (par_draw(key, pos, n, count, out, threads, 0, 0, 4.0, st)) {
    g_par_ok.fetch_add(1);
    return true;
  }
  g_par_fallback.fetch_add(1);
  return false;
}
}  // namespace dppo

extern "C" int dppo_perm_targets_numpy_par(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                                           int32_t* out, int32_t threads, const int64_t* opts,
                                           int64_t* stats) {
  if (!key || !pos || !out || n < 0 || n > 0x7FFFFFFF || count < 0 || *pos < 0 || *pos > kN)
    return DPPO_EINVAL;
  int64_t st[24] = {0};
  const int64_t chunks = opts ? opts[0] : 0;
  const int64_t w_over = opts ? opts[1] : 0;
  const double w_mult = opts && opts[2] > 0 ? (double)opts[2] / 100.0 : 4.0;
  bool done = false;
  if (threads >= 2 && n >= 2 && count > 0 && cpu_ok()) {
    done = par_draw(key, pos, n, count, out, threads, chunks, w_over, w_mult, st);
    st[0] = done ? 1 : 2;
  }
  if (!done) {
    const int rc = dppo_perm_targets_serial(key, pos, n, count, out);
    if (rc) return rc;
  }
  if (stats) std::memcpy(stats, st, sizeof(st));
  return DPPO_OK;
}

extern "C" int dppo_perm_par_stats(int64_t* out3) {
  if (!out3) return DPPO_EINVAL;
  out3[0] = g_par_calls.load();
  out3[1] = g_par_ok.load();
  out3[2] = g_par_fallback.load();
  return DPPO_OK;
}
