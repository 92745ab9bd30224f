#!/usr/bin/env python3
"""Scaling cap of the reference-exact multi-GPU mode (cfg.global_minibatches = True) at BASELINE
configs[4] (65,536 CartPole envs in total, strong scaling): every rank draws the reference's E
permutations of the GLOBAL batch (T x 65,536 = 8.4 M samples, E = 4: 33.5 M Fisher-Yates targets,
ppo.py:252-255) and resolves them on its device, while its share of the learn shrinks as 1/world.

For world = 1, 2, 4, 8:
* host draw per learn: the serial accept scan (perm.cpp) and the parallel speculative draw
  (permpar.cpp, DPPO_PERM_PAR_THREADS threads; what dppo_perm_targets_numpy runs), median of 5
  isolated draws, and of 10 chained ones (back to back, as a host-bound learn draws);
* on a GPU box: the device time per learn of one rank's share (T x 65,536/world envs, local
  minibatches, the same kernels) plus that rank's global-minibatch member lists from the swap
  targets (dppo_global_minibatch_lists: bucket build over all E x 8.4 M targets, the walk of the
  rank's own samples, the ordered selection); at world 1 the whole-permutation resolution.
The look-ahead drafts overlap the draw with the device, so a learn takes
max(draw, share + resolution); the cap is device(1) / that.

    python tools/gmb_cap.py [--no-gpu] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))


def host_draw_ms(n, epochs=4, reps=5, threads=1, chained=False):
    """Median ms of one draw of the learn's targets.  chained: each draw starts from the previous
    one's final state, back to back (the look-ahead drafts of a host-bound learn: the draw
    threads never rest, and the sustained load runs slower than isolated draws on the box)."""
    from diamond import _native as N
    out = np.empty(n * epochs, np.int32)
    ts = []
    key, pos, _ = N.mt_state(np.random.RandomState(42))
    for r in range(reps + 1):
        if not chained:
            key, pos, _ = N.mt_state(np.random.RandomState(42 + r))
        t0 = time.perf_counter()
        pos, _ = N.perm_targets_numpy_par(key, pos, n, epochs, out, threads)
        if r:  # the first draw is a warm-up (buffers, jump polynomials)
            ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def global_lists_ms(world, reps=5):
    """Device time of one rank's global-minibatch member lists at configs[4] over `world` ranks
    (dppo_global_minibatch_lists: bucket build over all 4 x 8.4 M targets, the walk of this
    rank's 1/world of the samples, the ordered selection), HIP events on the kernels."""
    import torch
    from diamond import _native as N
    T, Ng, E, M = 128, 65536, 4, 8
    Nl = Ng // world
    h = N.Handle(0, N.Dims(T, Nl, 4, 2, 0, 64, E, M, world, 0, 1))
    key, pos, _ = N.mt_state(np.random.RandomState(7))
    tg = np.empty(E * T * Ng, np.int32)
    N.perm_targets_numpy(key, pos, T * Ng, E, tg)
    dev = torch.device("cuda", 0)
    td = torch.from_numpy(tg).to(dev)
    local = torch.empty(E * T * Nl, dtype=torch.int32, device=dev)
    seg = torch.empty(E * (M + 1), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    call = lambda: N.check(h.lib.dppo_global_minibatch_lists(h.h, td.data_ptr(), local.data_ptr(),
                                                             seg.data_ptr(), s),
                           "dppo_global_minibatch_lists")
    call()
    torch.cuda.synchronize(dev)
    h.set_timing(True)
    for _ in range(reps):
        call()
    ms, cnt = h.timing()["perm"]
    h.set_timing(False)
    h.close()
    return ms / cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    T, Ng = 128, 65536
    threads = int(os.environ.get("DPPO_PERM_PAR_THREADS", "12"))
    draw_serial = host_draw_ms(T * Ng)
    draw_par = host_draw_ms(T * Ng, threads=threads)
    draw_chain = host_draw_ms(T * Ng, reps=10, threads=threads, chained=True)
    dev, resolve = {}, None
    if not a.no_gpu:
        import torch
        import bench
        device = torch.device("cuda", 0)
        for world in (1, 2, 4, 8):
            name = f"c5_share{world}"
            bench.CONFIGS[name] = ("CartPole-shaped PPO, one rank's share of 65,536 envs", T,
                                   Ng // world, 4, 2, False, 0.02, 0.005, "weak")
            r = bench.run_config(name, 1, 0, None, device, a.steps, 2)
            dev[world] = r["device_ms_per_step"]
            if world == 1:  # the one-GPU learn resolves all 4 x 8.4 M targets on the device
                k = r["kernels"].get("perm")
                resolve = {1: k["ms_total"] / a.steps if k else 0.0}
        for world in (2, 4, 8):
            resolve[world] = global_lists_ms(world)
    rows = []
    for world in (1, 2, 4, 8):
        row = {"world": world, "host_draw_ms_serial": round(draw_serial, 2),
               "host_draw_ms_parallel": round(draw_par, 2),
               "host_draw_ms_parallel_chained": round(draw_chain, 2), "draw_threads": threads,
               "global_samples": T * Ng, "targets_drawn": 4 * T * Ng}
        if dev:
            share = dev[world] - (resolve[1] if world == 1 else 0.0)
            rdev = share + resolve[world]  # each rank: its share + its global member lists
            row["device_ms_share_local"] = round(share, 3)
            row["device_ms_global_lists"] = round(resolve[world], 3)
            row["device_ms_per_learn_global"] = round(rdev, 3)
            for tag, draw in (("serial", draw_serial), ("parallel", draw_par),
                              ("parallel_chained", draw_chain)):
                bound = max(draw, rdev)
                row[f"learn_ms_bound_{tag}_draw"] = round(bound, 3)
                row[f"speedup_cap_{tag}_draw"] = round(dev[1] / bound, 2)
            row["host_bound_parallel_draw"] = draw_par > rdev
        rows.append(row)
    import platform
    cpu = platform.processor()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    res = {"cpu": cpu, "rows": rows}
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
