// Host synchronisation of a single-device loopback group (capi.cpp dppo_loopback_group): the
// generation barrier its ranks' host threads meet at around every exchange, and the "broken"
// state a timed-out barrier or a destroyed member leaves.  Plain C++ (no HIP), so the
// sanitizer builds (Makefile: tsan / asan) exercise exactly this code.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>

namespace dppo {

struct LoopSync {
  enum Result { kOk = 0, kBroken = 1, kTimeout = 2 };
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  // set when a barrier timed out or a member was destroyed: every member's exchange then fails
  // (arrival counts and peer buffers can no longer be trusted)
  bool broken = false;

  // Wait until all n ranks arrive (kOk), the group breaks (kBroken), or `timeout` passes
  // (kTimeout; the group is then broken for everyone).
  Result barrier(std::chrono::milliseconds timeout) {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return kBroken;
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return kOk;
    }
    if (!cv.wait_for(lk, timeout, [&] { return gen != g || broken; })) {
      broken = true;
      cv.notify_all();
      return kTimeout;
    }
    return gen == g ? kBroken : kOk;  // woken by a break, not by the last arriver
  }

  // Break the group (a member leaves): waiters return kBroken, later barriers fail at once.
  // Call with `mu` held.
  void break_locked() {
    broken = true;
    cv.notify_all();
  }
};

}  // namespace dppo
