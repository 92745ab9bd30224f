#!/usr/bin/env python3
"""Per-interval timing of the pipelined minibatch kernel (timing-only build).

    make -C diamond-ppo_amd variant NAME=trace DEFS=-DDPPO_PHASE_TRACE
    DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so python tools/phase_trace.py

Runs one dppo_minibatch_grad_f32 launch on the CartPole bench shape and prints, for each of the
NI barrier intervals of an interval set, the mean cycles each team spends issuing/draining its
phase work (arrival - previous release) and the mean interval length (release - release),
averaged over the steady-state sets of workgroup 0.
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
from diamond import _native as N  # noqa: E402

NAMES0 = ["L1", "L2", "La/Lc", "heads+loss", "head bwd + gather"]
NAMES1 = ["dZ2", "dZ1", "dW1", "dWa+dW2", "dWc"]
NI = len(NAMES0)  # barriers per interval set


def main():
    # PHASE_CONFIG: a bench.py config name (default cartpole4096)
    _, T, Nn, D, A, cont, pt, ptr, _ = bench.CONFIGS[os.environ.get("PHASE_CONFIG", "cartpole4096")]
    Nn = int(os.environ.get("ABL_N", Nn))
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=Nn, verbose=False)
    agent = Agent(None, cfg, envs=bench.SpecEnvs(D, A, cont))
    dev = agent.device
    ro, _ = bench.synth_rollout(T, Nn, D, A, cont, pt, ptr, 0, dev)
    agent.learn_device(ro)
    torch.cuda.synchronize()
    L = agent._learner
    h = L.handle
    hp = diamond.engine.hparams(cfg, cfg.lr, 0)
    mb = T * Nn // 8
    idx = torch.randperm(T * Nn, device=dev)[:mb].to(torch.int32)
    g = torch.zeros(L.flat.total, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    # WARM_LAUNCHES: back-to-back launches before the traced one, so that the in-kernel clock
    # below is the one the chip holds under sustained load (MI355X_MICROARCH.md, DVFS give-back)
    for _ in range(int(os.environ.get("WARM_LAUNCHES", "3"))):
        N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb,
                                              ctypes.byref(hp), g.data_ptr(), None, s))
    torch.cuda.synchronize()
    buf = np.zeros((128, 8, 2), np.int64)
    fn = h.lib.dppo_debug_phase_trace
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    arr, rel = buf[:, :, 0], buf[:, :, 1]
    nbar = int((rel[:, 0] != 0).sum())
    sets = nbar // NI
    print(f"barriers traced: {nbar} ({sets} interval sets)")
    work = np.zeros((nbar, 8))
    span = np.zeros(nbar)
    for k in range(1, nbar):
        work[k] = arr[k] - rel[k - 1]
        span[k] = rel[k].max() - rel[k - 1].max()
    steady = [k for k in range(nbar) if 1 <= k // NI < sets - 1]
    print(f"{'int':>3} {'team0 phase':>22} {'t0 cyc':>8} {'team1 phase':>10} {'t1 cyc':>8} "
          f"{'interval':>9}")
    tot = 0.0
    for i in range(NI):
        ks = [k for k in steady if k % NI == i]
        w0 = work[ks][:, :4].max(axis=1).mean()
        w1 = work[ks][:, 4:].max(axis=1).mean()
        sp = span[ks].mean()
        tot += sp
        print(f"{i:>3} {NAMES0[i]:>22} {w0:8.0f} {NAMES1[i]:>10} {w1:8.0f} {sp:9.0f}")
    print("per-wave phase cycles (waves 0-3 forward team, 4-7 backward team):")
    for i in range(NI):
        ks = [k for k in steady if k % NI == i]
        print(f"  int {i}: " + " ".join(f"{work[ks][:, w].mean():6.0f}" for w in range(8)))
    print(f"set total {tot:.0f} cycles; whole launch {rel[nbar - 1].max() - rel[0].min():.0f} "
          f"cycles from first to last barrier")
    if hasattr(h.lib, "dppo_debug_phase_edges"):
        ed = np.zeros((256, 6), np.int64)
        f3 = h.lib.dppo_debug_phase_edges
        f3.argtypes = [ctypes.c_void_p]
        assert f3(ed.ctypes.data) == 0
        g = min(256, (mb + 31) // 32)
        ed = ed[:g]
        pro, loop, epi = ed[:, 1] - ed[:, 0], ed[:, 2] - ed[:, 1], ed[:, 3] - ed[:, 2]
        rt0, rt1 = ed[:, 4], ed[:, 5]
        print(f"workgroups {g}: prologue {np.median(pro):.0f} cycles (max {pro.max()}), main loop "
              f"{np.median(loop):.0f} (max {loop.max()}), epilogue {np.median(epi):.0f} "
              f"(max {epi.max()}); start skew {(rt0.max() - rt0.min()) / 100:.2f} us, end skew "
              f"{(rt1.max() - rt1.min()) / 100:.2f} us, first start -> last end "
              f"{(rt1.max() - rt0.min()) / 100:.2f} us (s_memrealtime)")
        ghz = (ed[:, 3] - ed[:, 0]) / np.maximum(rt1 - rt0, 1) / 10.0
        print(f"in-kernel clock: median {np.median(ghz):.3f} GHz (min {ghz.min():.3f}, "
              f"max {ghz.max():.3f}) over workgroups")
    if hasattr(h.lib, "dppo_debug_heads_trace"):
        hb = np.zeros((128, 4), np.int64)
        f2 = h.lib.dppo_debug_heads_trace
        f2.argtypes = [ctypes.c_void_p]
        assert f2(hb.ctypes.data) == 0
        d = []
        for k in steady:
            if k % NI == 3 and hb[k, 0]:
                start = rel[k - 1, 0]  # wave 0's release from the previous barrier
                d.append((hb[k, 0] - start, hb[k, 1] - hb[k, 0], hb[k, 2] - hb[k, 1],
                          arr[k, 0] - hb[k, 2]))
        if d:
            m = np.mean(np.array(d), axis=0)
            print(f"heads+loss, wave 0: dots {m[0]:.0f}, softmax/logp {m[1]:.0f}, "
                  f"ratio/grads/DOUT {m[2]:.0f}, to barrier {m[3]:.0f} cycles")


if __name__ == "__main__":
    main()
