#!/usr/bin/env python3
"""Per-phase timing of the sample-split minibatch kernel (csrc/mbwave.hip; timing-only build).

    make -C diamond-ppo_amd variant NAME=trace DEFS=-DDPPO_PHASE_TRACE
    DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=20000 python tools/mbw_trace.py

Runs dppo_minibatch_grad_f32 launches on a bench.py shape (PHASE_CONFIG, default cartpole4096)
and prints, for workgroup 0, the mean cycles every wave spends in each phase of a 16-sample group
beside the phase's MFMA floor (v_mfma_f32_16x16x4_f32: 32 cycles each), then the prologue / main
loop / epilogue split over all workgroups and the in-kernel clock.
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

PHASES = ["L1", "L2", "La/Lc", "heads+loss", "head dW+bwd", "dh2 (+gather)", "dz2, dWa, dWc",
          "dh1, dW2, dW1"]


def main():
    _, T, Nn, D, A, cont, pt, ptr, _ = bench.CONFIGS[os.environ.get("PHASE_CONFIG", "cartpole4096")]
    # PHASE_N: the same shape with another number of envs (buffer footprint A/B)
    Nn = int(os.environ.get("PHASE_N", Nn))
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
    for _ in range(int(os.environ.get("WARM_LAUNCHES", "3"))):
        N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb,
                                              ctypes.byref(hp), g.data_ptr(), None, s))
    torch.cuda.synchronize()
    ph = np.zeros((4, 16, 10), np.int64)
    f = h.lib.dppo_debug_mbw_phase
    f.argtypes = [ctypes.c_void_p]
    assert f(ph.ctypes.data) == 0
    nkn = (D + 3) // 4
    nib = 1 if D <= 16 else 2
    floor = [4 * nkn, 64, 128, 0, 0, 128, 128, 128 + 16 * nib]
    ng = int((ph[0, :, 0] != 0).sum())
    print(f"groups traced per wave: {ng}")
    tot = 0.0
    print(f"{'phase':>16} " + " ".join(f"{'w' + str(w):>7}" for w in range(4)) +
          f" {'mean':>7} {'MFMA floor':>10}")
    for i in range(8):
        c = [(ph[w, 1:ng, i + 1] - ph[w, 1:ng, i]).mean() for w in range(4)]
        tot += np.mean(c)
        print(f"{PHASES[i]:>16} " + " ".join(f"{x:7.0f}" for x in c) +
              f" {np.mean(c):7.0f} {32 * floor[i]:10d}")
    gap = np.mean([(ph[w, 1:ng, 0] - ph[w, 0:ng - 1, 8]).mean() for w in range(4)])
    print(f"{'loop overhead':>16} {gap:7.0f}")
    print(f"group total {tot + gap:.0f} cycles, MFMA floor {32 * sum(floor)} "
          f"({32 * sum(floor) / (tot + gap):.2f})")
    ed = np.zeros((256, 6), np.int64)
    f3 = h.lib.dppo_debug_mbw_edges
    f3.argtypes = [ctypes.c_void_p]
    assert f3(ed.ctypes.data) == 0
    G = min(256, (mb + 63) // 64)
    ed = ed[:G]
    pro, loop, epi = ed[:, 1] - ed[:, 0], ed[:, 2] - ed[:, 1], ed[:, 3] - ed[:, 2]
    rt0, rt1 = ed[:, 4], ed[:, 5]
    print(f"workgroups {G}: prologue {np.median(pro):.0f} cycles (max {pro.max()}), main loop "
          f"{np.median(loop):.0f} (max {loop.max()}), epilogue {np.median(epi):.0f} "
          f"(max {epi.max()}); start skew {(rt0.max() - rt0.min()) / 100:.2f} us, end skew "
          f"{(rt1.max() - rt1.min()) / 100:.2f} us, first start -> last end "
          f"{(rt1.max() - rt0.min()) / 100:.2f} us")
    if hasattr(h.lib, "dppo_debug_mbw_epi"):
        ep = np.zeros(8, np.int64)
        f4 = h.lib.dppo_debug_mbw_epi
        f4.argtypes = [ctypes.c_void_p]
        assert f4(ep.ctypes.data) == 0
        names = ["put W2|Wa + small", "barrier", "sum W2|Wa + small", "barrier + put Wc|W1",
                 "barrier", "sum Wc|W1", "drain + barrier"]
        ep[7] = ed[0, 3]
        print("epilogue of workgroup 0 (cycles): " + ", ".join(
            f"{n} {ep[i + 1] - ep[i]}" for i, n in enumerate(names)) +
            f"; loop exit -> epilogue {ep[0] - ed[0, 2]}")
    ghz = (ed[:, 3] - ed[:, 0]) / np.maximum(rt1 - rt0, 1) / 10.0
    print(f"in-kernel clock: median {np.median(ghz):.3f} GHz (min {ghz.min():.3f}, "
          f"max {ghz.max():.3f})")


if __name__ == "__main__":
    main()
