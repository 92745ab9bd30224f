#!/usr/bin/env python3
"""Host draw of the reference-exact permutation targets at BASELINE configs[4] with global
minibatches (E = 4 permutations of T x 65,536 = 8,388,608 samples: ppo.py:252-255), serial
(perm.cpp) against the parallel speculative draw (permpar.cpp) at several thread counts.
Every parallel draw is checked bit for bit (targets, MT19937 key and pos) against the serial one.
--chain K also times K draws back to back, each from the previous one's final state (what the
learner's look-ahead drafts do when the draw is the bound: no idle time between draws, so the
helper threads' cores stay busy), the last one checked against K chained serial draws.

    python tools/perm_par_bench.py [--reps 5] [--threads 4,8,12,16] [--chain 8] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128 * 65536)
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", default="4,8,12,16")
    ap.add_argument("--chunks-per-thread", type=int, default=0,
                    help="chunks = this x threads (0: the library default, 2 per thread)")
    ap.add_argument("--chain", type=int, default=0)
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="idle time between chained draws (a device-bound learn's gaps)")
    ap.add_argument("--pinned", action="store_true",
                    help="draw into page-locked host memory (torch pin_memory, i.e. hipHostMalloc: "
                         "what the learner's upload slots are) instead of a NumPy array")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from diamond import _native as N
    n, E = a.n, a.epochs
    if a.pinned:
        import torch
        pin = torch.empty(n * E, dtype=torch.int32).pin_memory()
        got = pin.numpy()
    else:
        got = np.empty(n * E, np.int32)
        got.fill(0)
    rows = []
    serial_ms = []
    by_thr = {int(t): [] for t in a.threads.split(",")}
    # the serial references first (one per rep), then each thread count as its own block after
    # one untimed warm-up draw: a process keeps one configuration, and the chunk buffers (sized
    # on first use) are reused from call to call
    states = []
    for rep in range(a.reps):
        rs = np.random.RandomState(1234 + rep)
        rs.random_sample(rep * 37)  # a pos other than 624
        key, pos, _ = N.mt_state(rs)
        k1 = key.copy()
        r1 = np.empty(n * E, np.int32)
        r1.fill(0)  # pre-faulted: the timed draw writes into resident pages, as the parallel ones do
        t0 = time.perf_counter()
        p1, _ = N.perm_targets_numpy_par(k1, pos, n, E, r1, 1)
        serial_ms.append((time.perf_counter() - t0) * 1e3)
        states.append((key, pos, k1, p1, r1))
    for thr in by_thr:
        key, pos = states[0][0], states[0][1]
        ch = a.chunks_per_thread * thr
        N.perm_targets_numpy_par(key.copy(), pos, n, E, got, thr, chunks=ch)  # warm-up
        for rep, (key, pos, k1, p1, r1) in enumerate(states):
            k2 = key.copy()
            t0 = time.perf_counter()
            p2, st = N.perm_targets_numpy_par(k2, pos, n, E, got, thr, chunks=ch)
            ms = (time.perf_counter() - t0) * 1e3
            ok = bool(p1 == p2 and np.array_equal(k1, k2) and np.array_equal(r1, got))
            by_thr[thr].append(ms)
            st.update({"threads": thr, "rep": rep, "ms": round(ms, 3), "bit_exact": ok})
            rows.append(st)
            print(json.dumps(st), flush=True)
            if not ok:
                raise SystemExit(f"MISMATCH at threads={thr} rep={rep}")
    chained = {}
    if a.chain > 0:
        key0, pos0 = states[0][0], states[0][1]
        kc, pc = key0.copy(), pos0
        ref = np.zeros(n * E, np.int32)
        for _ in range(a.chain):
            pc, _ = N.perm_targets_numpy_par(kc, pc, n, E, ref, 1)
        for thr in by_thr:
            ch = a.chunks_per_thread * thr
            kk, pp = key0.copy(), pos0
            ts = []
            for _ in range(a.chain):
                if a.gap_ms > 0:
                    time.sleep(a.gap_ms * 1e-3)
                t0 = time.perf_counter()
                pp, _ = N.perm_targets_numpy_par(kk, pp, n, E, got, thr, chunks=ch)
                ts.append((time.perf_counter() - t0) * 1e3)
            ok = bool(pp == pc and np.array_equal(kk, kc) and np.array_equal(got, ref))
            if not ok:
                raise SystemExit(f"chained MISMATCH at threads={thr}")
            chained[thr] = [round(t, 3) for t in ts]
            print(json.dumps({"threads": thr, "chained_ms": chained[thr]}), flush=True)
    med = lambda x: round(float(np.median(x)), 3)
    summary = {"cpu": cpu_model(), "affinity_cpus": len(os.sched_getaffinity(0)),
               "output": "pinned" if a.pinned else "numpy",
               "n": n, "epochs": E, "targets": E * (n - 1),
               "serial_ms_median": med(serial_ms),
               "parallel_ms_median": {t: med(v) for t, v in by_thr.items()},
               "parallel_ms_min": {t: round(min(v), 3) for t, v in by_thr.items()},
               "fallbacks": sum(1 for r in rows if r["path"] != 1),
               "all_bit_exact": all(r["bit_exact"] for r in rows)}
    if chained:
        summary["gap_ms"] = a.gap_ms
        summary["chained_ms_median"] = {t: med(v[1:]) for t, v in chained.items()}
        summary["chained_ms_min"] = {t: round(min(v[1:]), 3) for t, v in chained.items()}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": summary, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
