#!/usr/bin/env python3
"""Scaling cap of the reference-exact multi-GPU mode (cfg.global_minibatches = True) at BASELINE
configs[4] (65,536 CartPole envs in total, strong scaling): every rank draws the reference's E
permutations of the GLOBAL batch (T x 65,536 = 8.4 M samples, E = 4: 33.5 M Fisher-Yates targets,
one sequential MT19937 accept scan -- ppo.py:252-255) while its device share shrinks as 1/world.

For world = 1, 2, 4, 8: the host draw time per learn (dppo_perm_targets_numpy, the draw the
device-shuffle path uses at these sizes; median of 3) and -- on a GPU box -- the device time per
learn of one rank's share (T x 65,536/world envs, local minibatches, the same kernels).  The
look-ahead drafts overlap the draws with the device, so a learn takes max(draw, device); the
cap is device(1) / max(draw, device(world)).

    python tools/gmb_cap.py [--no-gpu]
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


def host_draw_ms(n, epochs=4, reps=3):
    from diamond import _native as N
    out = np.empty(n * epochs, np.int32)
    ts = []
    for r in range(reps):
        rs = np.random.RandomState(42 + r)
        key, pos, _ = N.mt_state(rs)
        t0 = time.perf_counter()
        N.perm_targets_numpy(key, pos, n, epochs, out)
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    T, Ng = 128, 65536
    draw = host_draw_ms(T * Ng)
    dev = {}
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
    rows = []
    for world in (1, 2, 4, 8):
        row = {"world": world, "host_draw_ms_per_learn": round(draw, 2),
               "global_samples": T * Ng, "targets_drawn": 4 * T * Ng}
        if dev:
            d = dev[world]
            row["device_ms_per_learn_per_rank"] = d
            row["learn_ms_bound"] = round(max(draw, d), 3)
            row["host_bound"] = draw > d
            row["speedup_cap_vs_1gpu"] = round(dev[1] / max(draw, d), 2)
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
    print(json.dumps({"cpu": cpu, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
