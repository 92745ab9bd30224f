#!/usr/bin/env python3
"""Per-parameter error of the first minibatch gradient vs the golden reference (debug aid)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "diamond-ppo_amd"), ROOT]
import test_gpu_parity as tp  # noqa: E402
import diamond  # noqa: E402
from diamond import _native as N  # noqa: E402

for name in ("cartpole_small", "lunar_medium", "cheetah_small"):
    z = tp.load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, _ = (int(x) for x in z["dims"])
    agent = tp.make_agent(z)
    L = agent._learner
    h = L.handle
    hp = diamond.engine.hparams(agent.cfg, agent.cfg.lr, 0)
    ro = diamond.engine.stage_experience(tp.experience(z, 0), tp.dev(), bool(cont))
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), L.flat.flat.data_ptr(),
                                   ctypes.byref(hp), None, tp.stream()))
    B = T * Nn
    mb = B // agent.cfg.num_minibatches
    idx = tp.t(z["perms"][0][:mb], torch.int32)
    g = torch.zeros(L.flat.total, device=tp.dev())
    loss4 = (ctypes.c_float * 4)()
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb,
                                          ctypes.byref(hp), g.data_ptr(), loss4, tp.stream()))
    torch.cuda.synchronize()
    gl = g.cpu().numpy()
    Lay = h.layout
    ref = z["grads"][0]
    o = 0
    names = [n for n, _ in agent.network.named_parameters()]
    print(name, "mb", mb, "loss", loss4[0], z["loss"][0])
    for i in range(Lay.count):
        got = gl[Lay.offset[i]:Lay.offset[i] + Lay.numel[i]]
        r = ref[o:o + Lay.numel[i]]
        o += Lay.numel[i]
        err = np.abs(got - r).max()
        j = int(np.abs(got - r).argmax())
        print(f"  {names[i]:28s} n={Lay.numel[i]:5d} maxerr {err:.3e} scale {np.abs(r).max():.3e} "
              f"at {j}: got {got[j]:.6e} ref {r[j]:.6e}")

# decode the wrong elements of the hidden matrices of the last discrete case
for name in ("cartpole_small",):
    z = tp.load_golden(f"learn_{name}.npz")
    agent = tp.make_agent(z)
    L = agent._learner
    h = L.handle
    T, Nn, D, A, cont, _ = (int(x) for x in z["dims"])
    hp = diamond.engine.hparams(agent.cfg, agent.cfg.lr, 0)
    ro = diamond.engine.stage_experience(tp.experience(z, 0), tp.dev(), bool(cont))
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), L.flat.flat.data_ptr(),
                                   ctypes.byref(hp), None, tp.stream()))
    mb = T * Nn // agent.cfg.num_minibatches
    idx = tp.t(z["perms"][0][:mb], torch.int32)
    g = torch.zeros(L.flat.total, device=tp.dev())
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb,
                                          ctypes.byref(hp), g.data_ptr(), None, tp.stream()))
    torch.cuda.synchronize()
    gl = g.cpu().numpy()
    Lay = h.layout
    ref = z["grads"][0]
    o = 0
    for i in range(Lay.count):
        n = Lay.numel[i]
        if n == 4096:
            got, r = gl[Lay.offset[i]:Lay.offset[i] + n], ref[o:o + n]
            bad = np.nonzero(np.abs(got - r) > 1e-5)[0]
            print(f"param {i}: {len(bad)} wrong")
            from collections import Counter
            cq = Counter()
            for e in bad:
                row, col = divmod(int(e), 64)
                q, rem = divmod(row, 16)
                v, ob = divmod(rem, 4)
                rr, ib = divmod(col, 4)
                cq[(q, v, ob, ib)] += 1
            print("  (q, v, ob, ib) -> count of r:", sorted(cq.items())[:40])
        o += n
