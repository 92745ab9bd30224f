#!/usr/bin/env python3
"""perm_numpy called from a dedicated host thread (as the learn() draft worker does), E x n."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
from diamond import _native as N  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 524288
E = 4
out = np.empty(E * n, np.int32)
np.random.seed(42)
ts = []


def work():
    for _ in range(20):
        key, pos, _ = N.mt_state()
        t0 = time.perf_counter()
        N.perm_numpy(key, pos, n, E, out)
        ts.append(time.perf_counter() - t0)
        time.sleep(0.002)


th = threading.Thread(target=work)
th.start()
th.join()
print(f"perm_numpy from a draft thread: min {min(ts) * 1e3:.3f} ms, median "
      f"{np.median(ts) * 1e3:.3f} ms, {E}x{n} (2 ms idle between calls)")
