#!/usr/bin/env python3
"""Timeline of the single-launch slab reduction + clip + Adam kernel (csrc/optim.hip
reduce_adam_kernel; timing-only build).

    make -C diamond-ppo_amd variant-optim NAME=ratrace DEFS=-DDPPO_RA_TRACE
    DPPO_LIB=diamond-ppo_amd/build/libdppo_ratrace.so python tools/ra_trace.py

Runs learn() on a bench.py shape (PHASE_CONFIG, default cartpole4096) and prints, for the last
reduce_adam launch, every block's s_memrealtime stamps (100 MHz) relative to the earliest block
entry: entry, slabs summed, gradient + squares published (drained), fan-in released, Adam stores
drained.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import diamond  # noqa: E402

STAMPS = ["entry", "slabs summed", "published", "released", "adam drained"]


def main():
    _, T, Nn, D, A, cont, pt, ptr, _ = bench.CONFIGS[os.environ.get("PHASE_CONFIG", "cartpole4096")]
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=Nn, verbose=False)
    agent = Agent(None, cfg, envs=bench.SpecEnvs(D, A, cont))
    ro, _ = bench.synth_rollout(T, Nn, D, A, cont, pt, ptr, 0, agent.device)
    for _ in range(int(os.environ.get("WARM_LEARNS", "5"))):
        agent.learn_device(ro)
    torch.cuda.synchronize()
    h = agent._learner.handle
    ed = np.zeros((512, 5), np.int64)
    f = h.lib.dppo_debug_ra_edges
    f.argtypes = [ctypes.c_void_p]
    assert f(ed.ctypes.data) == 0
    nb = int((ed[:, 0] != 0).sum())
    ed = ed[:nb]
    t0 = ed[:, 0].min()
    rel = (ed - t0) / 100.0  # us
    print(f"blocks {nb}; times in us from the first block entry")
    print(f"{'stamp':>14} {'min':>7} {'median':>7} {'max':>7}")
    for i, n in enumerate(STAMPS):
        c = rel[:, i]
        c = c[ed[:, i] != 0]
        if len(c):
            print(f"{n:>14} {c.min():7.2f} {np.median(c):7.2f} {c.max():7.2f}")
    print("per-block phase medians (us): " + ", ".join(
        f"{STAMPS[i]}->{STAMPS[i + 1]} {np.median(rel[:, i + 1] - rel[:, i]):.2f}"
        for i in range(4)))


if __name__ == "__main__":
    main()
