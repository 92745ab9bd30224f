// Host-code stress test for the sanitizer builds (diamond-ppo_amd/Makefile: `make tsan`,
// `make asan`).  Test infrastructure only.  Exercises, with real threads:
//  * perm.cpp -- the permutation draws the learn() look-ahead runs: blocking draws from several
//    threads at once, chained asynchronous drafts (dppo_perm_numpy_async from a "draft thread",
//    their tickets waited and their buffers read on the "launching thread", exactly the engine's
//    protocol), the pinned swap pool, the producer ring of MT19937 blocks, scratch recycling;
//    results checked against a plain sequential restatement (draw targets, then the swap loop);
//  * loop_sync.h -- the loopback group's generation barrier: many rounds with n threads, a break
//    while ranks wait, a timed-out barrier.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "dppo.h"
#include "loop_sync.h"

namespace {

int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

// MT19937 init_genrand(seed) key (numpy RandomState(seed) state with pos = 624)
void seed_key(uint32_t seed, uint32_t* key) {
  key[0] = seed;
  for (int i = 1; i < 624; ++i) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + i;
}

// sequential reference: targets from dppo_perm_targets_numpy, then the Fisher-Yates swap loop
void reference(uint32_t seed, int64_t n, int count, std::vector<int32_t>& out, uint32_t* key_out,
               int32_t* pos_out) {
  uint32_t key[624];
  seed_key(seed, key);
  int32_t pos = 624;
  std::vector<int32_t> tg((size_t)(n * count));
  CHECK(dppo_perm_targets_numpy(key, &pos, n, count, tg.data()) == 0);
  out.resize((size_t)(n * count));
  for (int c = 0; c < count; ++c) {
    int32_t* a = out.data() + (int64_t)c * n;
    const int32_t* j = tg.data() + (int64_t)c * n;
    for (int64_t k = 0; k < n; ++k) a[k] = (int32_t)k;
    for (int64_t k = n - 1; k >= 1; --k) std::swap(a[k], a[j[k]]);
  }
  std::memcpy(key_out, key, sizeof(key));
  *pos_out = pos;
}

void test_concurrent_blocking_draws() {
  const int64_t n = (1 << 16) + 7;
  const int count = 4;
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t) {
    th.emplace_back([t, n, count] {
      for (int rep = 0; rep < 3; ++rep) {
        const uint32_t seed = 100 + 10 * t + rep;
        std::vector<int32_t> ref;
        uint32_t rkey[624];
        int32_t rpos;
        reference(seed, n, count, ref, rkey, &rpos);
        uint32_t key[624];
        seed_key(seed, key);
        int32_t pos = 624;
        std::vector<int32_t> out((size_t)(n * count));
        CHECK(dppo_perm_numpy(key, &pos, n, count, out.data()) == 0);
        CHECK(out == ref);
        CHECK(std::memcmp(key, rkey, sizeof(key)) == 0 && pos == rpos);
      }
    });
  }
  for (auto& x : th) x.join();
}

// The engine's look-ahead: a draft thread chains async drafts (each from the previous one's
// returned state) into rotating buffers; the launching thread waits each ticket, then reads.
void test_chained_async_drafts() {
  const int64_t n = 1 << 18;  // n * count >= 2^20: the producer ring runs
  const int count = 4;
  const int drafts = 5;
  std::vector<std::vector<int32_t>> bufs(3, std::vector<int32_t>((size_t)(n * count)));
  std::vector<void*> tickets(drafts, nullptr);
  std::vector<int> slot_of(drafts);
  std::atomic<int> ready{0};
  uint32_t key[624];
  seed_key(9, key);
  int32_t pos = 624;
  std::atomic<int> consumed{0};
  std::thread draft([&] {
    for (int d = 0; d < drafts; ++d) {
      while (d - consumed.load() >= 2) std::this_thread::yield();  // two drafts in flight
      slot_of[d] = d % 3;
      void* t = nullptr;
      CHECK(dppo_perm_numpy_async(key, &pos, n, count, bufs[d % 3].data(), &t) == 0);
      tickets[d] = t;
      ready.store(d + 1, std::memory_order_release);
    }
  });
  // reference stream: the same draws back to back
  uint32_t rkey[624];
  seed_key(9, rkey);
  int32_t rpos = 624;
  std::vector<int32_t> ref((size_t)(n * count));
  for (int d = 0; d < drafts; ++d) {
    while (ready.load(std::memory_order_acquire) <= d) std::this_thread::yield();
    CHECK(dppo_perm_wait(tickets[d]) == 0);
    CHECK(dppo_perm_numpy(rkey, &rpos, n, count, ref.data()) == 0);
    CHECK(bufs[slot_of[d]] == ref);
    consumed.store(d + 1);
  }
  draft.join();
  CHECK(std::memcmp(key, rkey, sizeof(key)) == 0 && pos == rpos);
}

// The parallel speculative draw (permpar.cpp) from several threads at once: the shared worker
// pool, the chunk-buffer free list, a forced fallback (tiny near-miss band); every result equal
// to the serial draw, generator state included.
void test_parallel_draws() {
  const int64_t n = (1 << 16) + 3;
  const int count = 3;
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t) {
    th.emplace_back([t, n, count] {
      for (int rep = 0; rep < 2; ++rep) {
        const uint32_t seed = 700 + 10 * t + rep;
        uint32_t rkey[624], key[624];
        seed_key(seed, rkey);
        std::memcpy(key, rkey, sizeof(key));
        int32_t rpos = 624, pos = 624;
        std::vector<int32_t> ref((size_t)(n * count)), out((size_t)(n * count));
        int64_t st[24];
        CHECK(dppo_perm_targets_numpy_par(rkey, &rpos, n, count, ref.data(), 1, nullptr, st) == 0);
        const int64_t opts[3] = {6, rep == 1 && t == 0 ? 8 : 0, 0};  // 6 chunks; one tiny band
        CHECK(dppo_perm_targets_numpy_par(key, &pos, n, count, out.data(), 4, opts, st) == 0);
        CHECK(st[0] == (rep == 1 && t == 0 ? 2 : 1));
        CHECK(out == ref);
        CHECK(std::memcmp(key, rkey, sizeof(key)) == 0 && pos == rpos);
      }
    });
  }
  for (auto& x : th) x.join();
}

void test_loop_barrier() {
  using dppo::LoopSync;
  {  // many generations, 4 ranks
    LoopSync g;
    g.n = 4;
    std::atomic<int> bad{0};
    std::vector<int> counter(4, 0);
    std::vector<std::thread> th;
    for (int r = 0; r < 4; ++r)
      th.emplace_back([&, r] {
        for (int it = 0; it < 2000; ++it) {
          counter[r] = it;
          if (g.barrier(std::chrono::seconds(30)) != LoopSync::kOk) ++bad;
          for (int q = 0; q < 4; ++q)  // every peer has written this round's value
            if (counter[q] < it) ++bad;
          if (g.barrier(std::chrono::seconds(30)) != LoopSync::kOk) ++bad;
        }
      });
    for (auto& x : th) x.join();
    CHECK(bad.load() == 0);
  }
  {  // a member leaves while the others wait: they return kBroken, later barriers too
    LoopSync g;
    g.n = 3;
    std::atomic<int> broken{0};
    std::vector<std::thread> th;
    for (int r = 0; r < 2; ++r)
      th.emplace_back([&] {
        if (g.barrier(std::chrono::seconds(30)) == LoopSync::kBroken) ++broken;
        if (g.barrier(std::chrono::seconds(30)) == LoopSync::kBroken) ++broken;
      });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    {
      std::lock_guard<std::mutex> lk(g.mu);
      g.break_locked();
    }
    for (auto& x : th) x.join();
    CHECK(broken.load() == 4);
  }
  {  // a rank never arrives: the waiters time out and the group is broken for everyone
    LoopSync g;
    g.n = 3;
    std::atomic<int> timeouts{0}, brokens{0};
    std::vector<std::thread> th;
    for (int r = 0; r < 2; ++r)
      th.emplace_back([&] {
        const auto res = g.barrier(std::chrono::milliseconds(100));
        if (res == LoopSync::kTimeout) ++timeouts;
        if (res == LoopSync::kBroken) ++brokens;
      });
    for (auto& x : th) x.join();
    CHECK(timeouts.load() >= 1 && timeouts.load() + brokens.load() == 2);
    CHECK(g.barrier(std::chrono::seconds(1)) == LoopSync::kBroken);
  }
}

}  // namespace

int main() {
  setenv("DPPO_PERM_PIN", "3", 1);  // the pinned swap pool in any container
  test_concurrent_blocking_draws();
  test_chained_async_drafts();
  test_parallel_draws();
  test_loop_barrier();
  int64_t st[3];
  dppo_perm_stats(st);
  CHECK(st[1] > 0 && st[2] > 0);  // the pool and the producer ring both ran
  std::printf("%s: %lld draws (%lld pooled, %lld with the ring), %d failures\n",
              g_fail ? "FAIL" : "OK", (long long)st[0], (long long)st[1], (long long)st[2], g_fail);
  return g_fail ? 1 : 0;
}
