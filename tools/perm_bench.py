#!/usr/bin/env python3
"""Host cost of the NumPy-exact minibatch permutations (ppo.py:254) at a given batch size:
full permutations (draws + Fisher-Yates swaps), the draws alone (swap targets), and NumPy."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
from diamond import _native as N  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
E = 4
out = np.empty(E * n, np.int32)
np.random.seed(42)
for cnt in (1, 2, E):
    for name, fn in (("perm_numpy", N.perm_numpy), ("perm_targets_numpy", N.perm_targets_numpy)):
        ts = []
        for _ in range(7):
            key, pos, _ = N.mt_state()
            t0 = time.perf_counter()
            fn(key, pos, n, cnt, out)
            ts.append(time.perf_counter() - t0)
        print(f"{name}: {min(ts) * 1e3:.3f} ms (min of 7), median {np.median(ts) * 1e3:.3f}, "
              f"{cnt}x{n}")
t0 = time.perf_counter()
for _ in range(E):
    np.random.permutation(n)
print(f"numpy permutation: {(time.perf_counter() - t0) * 1e3:.2f} ms")
try:
    print(open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0], os.cpu_count())
except Exception:
    pass
