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
// branch-light (AVX-512 groups of 16 draws); each epoch's swap chain runs on a persistent worker
// in the drawing thread's L3 domain while the next epoch is drawn (EPYC 9575F, 4 x 524,288:
// 1.3 ms against 2.25 ms on one thread).
// dppo_perm_targets_numpy stops after the draws: the swaps are resolved on the GPU instead
// (shuffle.hip), which takes the sequential swap chain off the host's critical path.

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
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
// (The sanitizer builds, DPPO_SANITIZE, compile one plain version: an ifunc resolver runs during
// relocation, before the sanitizer runtime is up, and its instrumented code crashes there.)
#ifdef DPPO_SANITIZE
#define DPPO_TWIST_CLONES
#else
#define DPPO_TWIST_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))
#endif
DPPO_TWIST_CLONES void twist_block(uint32_t* __restrict mt, uint32_t* __restrict out) {
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
  uint32_t out[kN];  // tempered outputs of the current block (when twisted in this thread)
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
// The MT19937 blocks the draws consume: twisted here (LocalBlocks) or by a producer thread
// running ahead (RingBlocks).  next() returns the next block's 624 tempered words.
struct LocalBlocks {
  MT& g;
  const uint32_t* first() const { return g.out; }
  const uint32_t* next() {
    twist_block(g.mt, g.out);
    return g.out;
  }
};

template <class Blocks>
const uint32_t* draw_targets_from(Blocks& src, const uint32_t* blk, int& pos, int64_t n,
                                  int32_t count, int32_t* __restrict out) {
  int opos = pos;
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
          blk = src.next();
          opos = 0;
        }
        if (simd && i >= lo + 15) {
          opos += (int)draw_groups_avx512(blk + opos, (uint32_t)(kN - opos), mask, i, lo, j);
          if (opos >= kN || i < lo) continue;
        }
        const uint32_t* __restrict o = blk + opos;
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
  pos = opos;
  return blk;
}

void draw_targets(MT& g, int64_t n, int32_t count, int32_t* __restrict out) {
  LocalBlocks src{g};
  draw_targets_from(src, src.first(), g.pos, n, count, out);
}

// numpy's state key is the untempered block: tempering is a bijection, so the key of a block
// that was twisted in another thread is recovered from its tempered words.
inline uint32_t untemper(uint32_t y) {
  y ^= y >> 18;
  y ^= (y << 15) & 0xEFC60000u;
  uint32_t x = y;
  for (int k = 0; k < 4; ++k) x = y ^ ((x << 7) & 0x9D2C5680u);
  y = x;
  return y ^ (y >> 11) ^ (y >> 22);
}

// A producer thread twists the blocks ahead of the drawing thread into a single-producer /
// single-consumer ring (the twist is ~37 % of the draw time): the draws then cost the accept
// scan alone.  A slot is released when the consumer moves past it.
class RingBlocks {
 public:
  explicit RingBlocks(const uint32_t* key, const cpu_set_t* cpus) {
    std::memcpy(mt_, key, sizeof(mt_));
    th_ = std::thread([this] { produce(); });
    if (cpus) pthread_setaffinity_np(th_.native_handle(), sizeof(*cpus), cpus);
  }
  ~RingBlocks() {
    stop_.store(true, std::memory_order_relaxed);
    th_.join();
  }
  const uint32_t* next() {
    if (held_) tail_.store(tail_.load(std::memory_order_relaxed) + 1, std::memory_order_release);
    held_ = true;
    const uint64_t t = tail_.load(std::memory_order_relaxed);
    while (head_.load(std::memory_order_acquire) == t) _mm_pause();
    return slots_[t % kCap];
  }

 private:
  static constexpr int kCap = 32;
  void produce() {
    uint64_t h = 0;
    while (!stop_.load(std::memory_order_relaxed)) {
      if (h - tail_.load(std::memory_order_acquire) >= (uint64_t)kCap) {
        _mm_pause();
        continue;
      }
      twist_block(mt_, slots_[h % kCap]);
      head_.store(++h, std::memory_order_release);
    }
  }
  alignas(64) uint32_t slots_[kCap][kN];
  uint32_t mt_[kN];
  alignas(64) std::atomic<uint64_t> head_{0};
  alignas(64) std::atomic<uint64_t> tail_{0};
  std::atomic<bool> stop_{false};
  bool held_ = false;
  std::thread th_;
};

// a[0..n) = arange(n) shuffled by the Fisher-Yates targets j: the sequential swap loop for
// i = n-1 .. 1, with the target lines prefetched ahead.
void apply_swaps(int32_t* __restrict a, const int32_t* __restrict j, int64_t n) {
  for (int64_t k = 0; k < n; ++k) a[k] = (int32_t)k;
  constexpr int kAhead = 32;
  for (int64_t k = n - 1; k >= 1; --k) {
    // the targets stream in from the drawing thread's caches (another core, maybe another
    // L3): fetch their lines well ahead of the sequential walk
    if ((k & 15) == 0 && k >= 1024) __builtin_prefetch(j + k - 1024, 0, 3);
    if (k - kAhead >= 1) __builtin_prefetch(a + j[k - kAhead], 1, 3);
    const int32_t v = j[k];
    const int32_t t = a[k];
    a[k] = a[v];
    a[v] = t;
  }
}

// The allowed CPUs that share an L3 with `cpu`.
bool l3_of(int cpu, const cpu_set_t& allowed, cpu_set_t* out) {
  char path[96];
  std::snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list",
                cpu);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[512] = {0};
  const bool got = std::fgets(buf, sizeof(buf), f) != nullptr;
  std::fclose(f);
  if (!got) return false;
  CPU_ZERO(out);
  int count = 0;
  for (char* p = buf; *p;) {  // "a-b,c,d-e"
    char* e;
    const long a = std::strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    p = e;
    if (*p == '-') {
      b = std::strtol(p + 1, &e, 10);
      p = e;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (c >= 0 && CPU_ISSET(c, &allowed)) {
        CPU_SET(c, out);
        ++count;
      }
    while (*p == ',' || *p == '\n' || *p == ' ') ++p;
  }
  return count >= 2;
}

// The CPU the process's main thread last ran on (/proc/self/task/<pid>/stat field 39), or -1.
int main_thread_cpu() {
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/self/task/%d/stat", (int)getpid());
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  char buf[1024] = {0};
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');  // the command name may hold spaces
  if (!p) return -1;
  int field = 2;
  for (; *p && field < 39; ++p)
    if (*p == ' ') ++field;
  return *p ? std::atoi(p) : -1;
}

// Busy fraction of every CPU over a short window, from two reads of /proc/stat (host-wide counters:
// on a shared box they include the other tenants' load).  busy[c] < 0 where unknown.
bool cpu_busy(std::vector<double>* busy, int window_ms) {
  auto read = [](std::vector<std::pair<unsigned long long, unsigned long long>>* v) {
    FILE* f = std::fopen("/proc/stat", "r");
    if (!f) return false;
    char line[512];
    v->assign(CPU_SETSIZE, {0ull, 0ull});
    while (std::fgets(line, sizeof(line), f)) {
      int cpu = -1;
      unsigned long long x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (std::sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, x, x + 1,
                      x + 2, x + 3, x + 4, x + 5, x + 6, x + 7) >= 5 &&
          cpu >= 0 && cpu < CPU_SETSIZE) {
        unsigned long long tot = 0;
        for (unsigned long long y : x) tot += y;
        (*v)[cpu] = {tot, x[3] + x[4]};  // (total, idle + iowait)
      }
    }
    std::fclose(f);
    return true;
  };
  std::vector<std::pair<unsigned long long, unsigned long long>> a, b;
  if (!read(&a)) return false;
  std::this_thread::sleep_for(std::chrono::milliseconds(window_ms));
  if (!read(&b)) return false;
  busy->assign(CPU_SETSIZE, -1.0);
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    const unsigned long long dt = b[c].first - a[c].first, di = b[c].second - a[c].second;
    if (b[c].first > a[c].first) (*busy)[c] = 1.0 - (double)di / (double)dt;
  }
  return true;
}

double domain_busy(const cpu_set_t& d, const std::vector<double>& busy) {
  double s = 0.0;
  int n = 0;
  for (int c = 0; c < CPU_SETSIZE && c < (int)busy.size(); ++c)
    if (CPU_ISSET(c, &d) && busy[c] >= 0.0) {
      s += busy[c];
      ++n;
    }
  return n ? s / n : 0.0;
}

std::atomic<int> g_dom_first{-1};       // first CPU of the swap pool's L3 domain
std::atomic<int> g_dom_busy_pct{-1};    // its busy fraction when chosen (%)
std::atomic<int> g_repins{0};

// Where the swap workers (and the drawing thread) run.  The swap chain of an epoch reads the
// targets the drawing thread just wrote, so they share one L3 (EPYC 9575F, 4 x 524,288: 1.3 ms
// in one L3 against 3-4 ms placed freely and 2.25 ms on one thread).  And that L3 is not the
// main thread's where the process may use another: the main thread and the HIP runtime's threads
// launch the learn's ~70 kernels.  mode 1: the L3 of the calling thread; mode 2 (default): an L3
// other than the main thread's, else the caller's.
bool l3_domain(int mode, cpu_set_t* out) {
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  if (mode == 3) {  // every allowed CPU (tests: the pooled path without a cache topology)
    *out = allowed;
    return CPU_COUNT(&allowed) >= 1;
  }
  const int home = sched_getcpu();
  if (mode == 1) return home >= 0 && l3_of(home, allowed, out) && CPU_ISSET(home, out);
  const int mcpu = main_thread_cpu();
  cpu_set_t mine;
  const bool have_main = mcpu >= 0 && l3_of(mcpu, allowed, &mine);
  // the candidate L3 domains (>= 4 allowed CPUs, not the main thread's), in CPU order
  std::vector<cpu_set_t> doms;
  cpu_set_t seen;
  CPU_ZERO(&seen);
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &allowed) || CPU_ISSET(c, &seen)) continue;
    cpu_set_t d;
    if (!l3_of(c, allowed, &d)) continue;
    CPU_OR(&seen, &seen, &d);
    if ((have_main && CPU_ISSET(c, &mine)) || CPU_COUNT(&d) < 4) continue;
    doms.push_back(d);
  }
  if (!doms.empty()) {
    // Busy domains last (round 6: on the shared GPU box a draw pinned to a CCD that other tenants
    // kept busy ran 6x slower -- 13.2 ms per learn instead of 2.2, the whole C3 learn host-bound
    // at 75 M env-steps/s instead of 286 M).  CPU order stays the preference among the domains
    // under DPPO_PERM_BUSY_MAX (default 30 %) busy: a first version that sorted every domain by
    // load moved the pool off its usual CCD over fractions of a percent and the same learn lost
    // 0.7 ms to slower swaps there (memory placement), so only a busy domain is passed over; the
    // busy ones follow, least busy first.  DPPO_PERM_BY_LOAD=0: CPU order only.
    static const bool by_load = [] {
      const char* e = std::getenv("DPPO_PERM_BY_LOAD");
      return !(e && e[0] == '0');
    }();
    static const double busy_max = [] {
      const char* e = std::getenv("DPPO_PERM_BUSY_MAX");
      return e ? std::atof(e) / 100.0 : 0.30;
    }();
    std::vector<double> busy;
    std::vector<double> load(doms.size(), 0.0);
    if (by_load && doms.size() > 1 && cpu_busy(&busy, 25)) {
      for (size_t i = 0; i < doms.size(); ++i) load[i] = domain_busy(doms[i], busy);
      std::vector<size_t> order(doms.size());
      for (size_t i = 0; i < order.size(); ++i) order[i] = i;
      std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
        const bool bx = load[x] >= busy_max, by = load[y] >= busy_max;
        if (bx != by) return by;          // idle enough first, in CPU order
        return bx && load[x] < load[y];   // then the busy ones, least busy first
      });
      std::vector<cpu_set_t> sorted;
      std::vector<double> sl;
      for (size_t i : order) {
        sorted.push_back(doms[i]);
        sl.push_back(load[i]);
      }
      doms.swap(sorted);
      load.swap(sl);
    }
    // one process per GPU (torchrun's LOCAL_RANK): spread the ranks' pools over the domains
    // instead of stacking every rank's draft and swap threads on the first one
    const char* lr = std::getenv("LOCAL_RANK");
    const size_t k = lr ? (size_t)std::max(0, std::atoi(lr)) % doms.size() : 0;
    *out = doms[k];
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, out)) {
        g_dom_first.store(c);
        break;
      }
    g_dom_busy_pct.store((int)(100.0 * load[k] + 0.5));
    return true;
  }
  // every allowed CPU shares the main thread's L3 (a cpuset of one CCD): the caller's L3 still
  // beats an unpinned pool or one thread (measured equal to mode 2 once the slot waits moved off
  // the draft thread)
  const bool ok = home >= 0 && l3_of(home, allowed, out) && CPU_ISSET(home, out);
  if (ok)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, out)) {
        g_dom_first.store(c);
        break;
      }
  return ok;
}

// Persistent swap workers: epoch c's swap chain runs while epoch c+1 is drawn, without a thread
// start (~50 us) or a fresh 2 MiB target buffer (~500 first-touch page faults) per epoch.  The
// pool is never torn down (idle workers wait on a condition variable); each call tracks its own
// jobs, so concurrent callers (loopback ranks on host threads) share it safely.
class SwapPool {
 public:
  struct Batch {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
  };
  static SwapPool& get() {
    static SwapPool* p = new SwapPool();  // leaked on purpose: no join at process exit
    return *p;
  }
  void submit(Batch* b, int32_t* a, const int32_t* j, int64_t n) {
    {
      std::lock_guard<std::mutex> g(b->mu);
      ++b->left;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(Job{b, a, j, n});
      nq_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_one();
  }
  static void wait(Batch* b) {
    std::unique_lock<std::mutex> g(b->mu);
    b->cv.wait(g, [&] { return b->left == 0; });
  }

 private:
  struct Job {
    Batch* b;
    int32_t* a;
    const int32_t* j;
    int64_t n;
  };
  // Workers share the L3 domain of the thread that creates the pool; callers other than the
  // process's main thread move themselves into it (see pin_caller).
  SwapPool() {
    const char* e = std::getenv("DPPO_PERM_WORKERS");
    const int nw = e ? std::max(1, std::atoi(e)) : 3;
    const char* sp = std::getenv("DPPO_PERM_SPIN_MS");
    spin_ms_ = sp ? std::atoi(sp) : 0;
    const char* pe = std::getenv("DPPO_PERM_PIN");
    const int mode = pe ? std::atoi(pe) : 2;
    mode_ = mode;
    pinned_ = mode != 0 && l3_domain(mode, &l3_);
    for (int i = 0; i < nw; ++i) {
      std::thread t([this] { run(); });
      if (pinned_) pthread_setaffinity_np(t.native_handle(), sizeof(l3_), &l3_);
      t.detach();
    }
  }

 public:
  // A draft thread (not the main thread: its affinity would be inherited by every thread it
  // starts later) joins the workers' L3 domain, once.
  bool pinned() const { return pinned_; }
  // the pool's domain (a copy: repin() may replace it)
  bool cpus(cpu_set_t* out) {
    if (!pinned_) return false;
    std::lock_guard<std::mutex> g(dom_mu_);
    *out = l3_;
    return true;
  }
  void pin_caller() {
    static thread_local unsigned done = 0;  // the domain generation this thread is pinned to
    if (!pinned_) return;
    const unsigned gen = gen_.load(std::memory_order_acquire);
    if (done == gen + 1) return;
    done = gen + 1;
    if ((pid_t)syscall(SYS_gettid) != getpid()) {
      cpu_set_t d;
      cpus(&d);
      pthread_setaffinity_np(pthread_self(), sizeof(d), &d);
    }
  }
  // Choose the domain again by load (another tenant may have taken ours): the workers and the
  // pinned callers move at their next job.  Returns whether the domain changed.
  bool repin() {
    if (!pinned_ || mode_ != 2) return false;
    cpu_set_t d;
    if (!l3_domain(2, &d)) return false;
    std::lock_guard<std::mutex> g(dom_mu_);
    if (CPU_EQUAL(&d, &l3_)) return false;
    l3_ = d;
    gen_.fetch_add(1, std::memory_order_acq_rel);
    g_repins.fetch_add(1, std::memory_order_relaxed);
    return true;
  }

 private:
  void run() {
    for (;;) {
      Job job;
      // optional spin before sleeping (DPPO_PERM_SPIN_MS; off by default: it holds cores)
      const auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; nq_.load(std::memory_order_acquire) == 0; ++it) {
        _mm_pause();
        if ((it & 1023) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(spin_ms_))
          break;
      }
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return !q_.empty(); });
        job = q_.front();
        q_.pop_front();
        nq_.fetch_sub(1, std::memory_order_relaxed);
      }
      pin_caller();  // (a worker follows repin() at its next job)
      apply_swaps(job.a, job.j, job.n);
      std::lock_guard<std::mutex> g(job.b->mu);
      if (--job.b->left == 0) job.b->cv.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  std::atomic<int> nq_{0};
  int spin_ms_ = 0;
  int mode_ = 0;
  bool pinned_ = false;
  std::mutex dom_mu_;
  std::atomic<unsigned> gen_{0};
  cpu_set_t l3_;
};

bool bad_args(const uint32_t* key, const int32_t* pos, int64_t n, int32_t count,
              const int32_t* out) {
  return !key || !pos || !out || n < 0 || n > 0x7FFFFFFF || count < 0 || *pos < 0 || *pos > kN;
}

std::atomic<int64_t> g_targets_ringed{0};

}  // namespace

namespace dppo {
bool perm_targets_parallel(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out);
}

// The serial draw (permpar.cpp falls back to it).
int dppo_perm_targets_serial(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out) {
  if (bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  MT g;
  g.load(key, *pos);
  draw_targets(g, n, count, out);
  std::memcpy(key, g.mt, sizeof(g.mt));
  *pos = g.pos;
  return DPPO_OK;
}

extern "C" int dppo_perm_targets_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                                       int32_t* out) {
  if (bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  // large draws (C5's global minibatches: 4 x 8.4 M targets): the speculative chunked scan of
  // permpar.cpp on DPPO_PERM_PAR_THREADS threads (default 12; 0 or 1 = this serial scan)
  if (dppo::perm_targets_parallel(key, pos, n, count, out)) return DPPO_OK;
  MT g;
  g.load(key, *pos);
  // DPPO_PERM_TARGETS_RING=1 (A/B only): a producer thread twists the MT19937 blocks ahead of
  // this accept scan.  Off by default: on the GPU box's EPYC 9575F the 4 x 8.4 M-target draw of
  // C5's global minibatches took 65 ms with the ring against 15.8 ms on one thread (the AVX-512
  // twist is cheap next to the scan, and the hand-off lines cost more than they save).
  static const int ring_mode = [] {
    const char* e = std::getenv("DPPO_PERM_TARGETS_RING");
    return e ? std::atoi(e) : 0;
  }();
  if (ring_mode && n * count >= (1 << 20)) {
    cpu_set_t dom;
    RingBlocks ring(g.mt, SwapPool::get().cpus(&dom) ? &dom : nullptr);
    int p = g.pos;
    const uint32_t* blk = draw_targets_from(ring, g.out, p, n, count, out);
    if (blk != g.out) {
      for (int k = 0; k < kN; ++k) key[k] = untemper(blk[k]);
    } else {
      std::memcpy(key, g.mt, sizeof(g.mt));
    }
    *pos = p;
    g_targets_ringed.fetch_add(1, std::memory_order_relaxed);
    return DPPO_OK;
  }
  draw_targets(g, n, count, out);
  std::memcpy(key, g.mt, sizeof(g.mt));
  *pos = g.pos;
  return DPPO_OK;
}

namespace {

// An in-flight permutation draw: the swaps still running on the pool and the target scratch they
// read.  Scratch buffers are recycled (a fresh 8 MiB buffer per call costs ~2,000 first-touch page
// faults), at most a few at a time: one per draft in flight.
struct PermTicket {
  SwapPool::Batch batch;
  std::vector<int32_t> scratch;
  bool pooled = false;
};
std::mutex g_scratch_mu;
std::vector<std::vector<int32_t>> g_scratch_free;
// calls of perm_start, of those on the swap pool, of those with the producer ring (dppo_perm_stats)
std::atomic<int64_t> g_calls{0}, g_pooled{0}, g_ringed{0};

std::vector<int32_t> take_scratch(size_t n) {
  std::lock_guard<std::mutex> g(g_scratch_mu);
  size_t best = g_scratch_free.size();  // the smallest buffer that fits
  for (size_t i = 0; i < g_scratch_free.size(); ++i)
    if (g_scratch_free[i].size() >= n &&
        (best == g_scratch_free.size() || g_scratch_free[i].size() < g_scratch_free[best].size()))
      best = i;
  if (best < g_scratch_free.size()) {
    std::vector<int32_t> v = std::move(g_scratch_free[best]);
    g_scratch_free.erase(g_scratch_free.begin() + (long)best);
    return v;
  }
  return std::vector<int32_t>(n);
}
void give_scratch(std::vector<int32_t>&& v) {
  std::lock_guard<std::mutex> g(g_scratch_mu);
  if (g_scratch_free.size() < 4) {
    g_scratch_free.push_back(std::move(v));
    return;
  }
  // full: a larger buffer replaces the smallest (a handle with a larger batch after a smaller
  // one otherwise allocated -- and zero-filled -- a fresh buffer on every call)
  size_t k = 0;
  for (size_t i = 1; i < g_scratch_free.size(); ++i)
    if (g_scratch_free[i].size() < g_scratch_free[k].size()) k = i;
  if (g_scratch_free[k].size() < v.size()) g_scratch_free[k] = std::move(v);
}

// Targets first (into the ticket's scratch), then the swaps into out -- the same state machine as
// numpy's fused loop.  The draws are one sequential MT19937 stream; the swaps of epoch c only need
// epoch c's targets, so at minibatch sizes they run on the pool while the next epoch is drawn,
// and the caller may start the NEXT draw (from the returned RNG state) before they finish.
int perm_start(uint32_t* key, int32_t* pos, int64_t n, int32_t count, int32_t* out,
               PermTicket* t) {
  MT g;
  g.load(key, *pos);
  static const int pool_mode = [] {
    const char* e = std::getenv("DPPO_PERM_POOL");
    return e ? std::atoi(e) : 1;
  }();
  // unpinned workers lose to one thread (see l3_domain): pool only inside one L3 domain
  t->pooled = pool_mode && n >= (1 << 16) && count > 1 && SwapPool::get().pinned();
  t->scratch = take_scratch((size_t)(n * count));
  if (t->pooled) SwapPool::get().pin_caller();
  // beside the pool, a producer thread twists the MT19937 blocks ahead of the draws
  static const int ring_mode = [] {
    const char* e = std::getenv("DPPO_PERM_RING");
    return e ? std::atoi(e) : 1;
  }();
  std::unique_ptr<RingBlocks> ring;
  cpu_set_t dom;
  if (t->pooled && ring_mode && n * count >= (1 << 20))
    ring.reset(new RingBlocks(g.mt, SwapPool::get().cpus(&dom) ? &dom : nullptr));
  g_calls.fetch_add(1, std::memory_order_relaxed);
  if (t->pooled) g_pooled.fetch_add(1, std::memory_order_relaxed);
  if (ring) g_ringed.fetch_add(1, std::memory_order_relaxed);
  LocalBlocks local{g};
  const uint32_t* blk = g.out;
  int p = g.pos;
  for (int32_t c = 0; c < count; ++c) {
    int32_t* j = t->scratch.data() + (int64_t)c * n;
    blk = ring ? draw_targets_from(*ring, blk, p, n, 1, j) : draw_targets_from(local, blk, p, n, 1, j);
    if (t->pooled)
      SwapPool::get().submit(&t->batch, out + (int64_t)c * n, j, n);
    else
      apply_swaps(out + (int64_t)c * n, j, n);
  }
  if (ring && blk != g.out) {
    for (int k = 0; k < kN; ++k) key[k] = untemper(blk[k]);
  } else {
    std::memcpy(key, g.mt, sizeof(g.mt));
  }
  *pos = p;
  return DPPO_OK;
}

void perm_finish(PermTicket* t) {
  if (t->pooled) SwapPool::wait(&t->batch);
  give_scratch(std::move(t->scratch));
  delete t;
}

}  // namespace

extern "C" int dppo_perm_numpy(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                               int32_t* out) {
  if (bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  PermTicket* t = new PermTicket();
  const int rc = perm_start(key, pos, n, count, out, t);
  perm_finish(t);
  return rc;
}

extern "C" int dppo_perm_numpy_async(uint32_t* key, int32_t* pos, int64_t n, int32_t count,
                                     int32_t* out, void** ticket) {
  if (!ticket || bad_args(key, pos, n, count, out)) return DPPO_EINVAL;
  PermTicket* t = new PermTicket();
  const int rc = perm_start(key, pos, n, count, out, t);
  *ticket = t;
  return rc;
}

extern "C" int dppo_perm_repin(int64_t* out4) {
  const bool moved = SwapPool::get().repin();
  if (out4) {
    out4[0] = moved ? 1 : 0;
    out4[1] = g_dom_first.load();
    out4[2] = g_dom_busy_pct.load();
    out4[3] = g_repins.load();
  }
  return DPPO_OK;
}

extern "C" int dppo_perm_domain(int64_t* out3) {
  if (!out3) return DPPO_EINVAL;
  (void)SwapPool::get();
  out3[0] = g_dom_first.load();
  out3[1] = g_dom_busy_pct.load();
  out3[2] = g_repins.load();
  return DPPO_OK;
}

extern "C" int dppo_perm_stats(int64_t* out3) {
  if (!out3) return DPPO_EINVAL;
  out3[0] = g_calls.load();
  out3[1] = g_pooled.load();
  out3[2] = g_ringed.load();
  return DPPO_OK;
}

extern "C" int dppo_perm_wait(void* ticket) {
  if (!ticket) return DPPO_EINVAL;
  perm_finish(static_cast<PermTicket*>(ticket));
  return DPPO_OK;
}
