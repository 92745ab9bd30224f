"""GPU parity of the minibatch gradient over a seeded sweep of network shapes.

Both minibatch kernels (csrc/mbwave.hip sample-split, csrc/mbstep.hip two-team; the dispatch is
csrc/common.h launch_mb / mbwave.hip mbw_supported) are instantiated per (action rows, Gaussian
head, input width) class.  This sweep draws 24 shapes from a fixed seed -- observation widths
1..32 (one or two 16-input column blocks, layer-1 k-steps 1..8), 1..8 actions, categorical and
Gaussian heads, minibatch sizes that leave partial 16-sample groups and idle waves / workgroups --
and checks one minibatch gradient through dppo_minibatch_grad_f32 against the NumPy oracle
(reference ppo.py:261-283, continuous_ppo.py:273-295) on the same records and indices, with the
bounds of tests/test_gpu_production.py: within 2e-5 * max|g| of the oracle evaluated in float64,
each tensor within 1e-4 of its own scale, the loss components within 2e-5.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from diamond import _native as N
from oracle import ppo_np as P

from gpu_helpers import H, dev, hparams, random_params, sample_split, stream, synth


def _shapes():
    rng = np.random.default_rng(20261016)
    out = []
    for i in range(24):
        D = int(rng.choice([1, 2, 3, 4, 5, 8, 11, 16, 17, 20, 24, 32]))
        A = int(rng.integers(1, 9))
        cont = bool(rng.integers(0, 2))
        if not cont and A == 1:
            A = 2  # a one-action categorical head is degenerate (log-prob 0, no gradient)
        T = int(rng.choice([8, 16, 24]))
        Nn = int(rng.choice([40, 64, 96, 160, 512]))
        M = int(rng.choice([1, 2, 4, 8]))
        while (T * Nn) % M:
            M //= 2
        ragged = int(rng.integers(0, 17))
        out.append((i, D, A, cont, T, Nn, M, ragged))
    return out


# One shape per head path of the sample-split kernel (mbwave.hip, round 3): head rows held in
# registers (<= 4 heads: 1-2 and 3-4 action rows, one or two input blocks), the heads and their
# back-propagation as MFMA tiles (5-8 categorical actions; 5-6 Gaussian actions on 17 inputs,
# HalfCheetah's X1 layout), each with a partial last 16-sample group.
_HEAD_SHAPES = [(4, 2, False), (3, 1, True), (8, 3, False), (8, 4, False), (11, 4, True),
                (20, 3, False), (16, 5, False), (8, 7, False), (16, 8, False), (17, 5, True),
                (17, 6, True),
                # 9-16 actions (the C-ABI's limit is 16): the two-team kernel's 16-head build
                (6, 12, False), (5, 10, True), (32, 16, False)]


@pytest.mark.parametrize("j,D,A,cont", [(j, *s) for j, s in enumerate(_HEAD_SHAPES)])
def test_minibatch_gradient_head_paths(j, D, A, cont):
    _check(100 + j, D, A, cont, 16, 96, 4, 5)


@pytest.mark.parametrize("i,D,A,cont,T,Nn,M,ragged", _shapes())
def test_minibatch_gradient_shape_sweep(i, D, A, cont, T, Nn, M, ragged):
    _check(i, D, A, cont, T, Nn, M, ragged)


def _check(i, D, A, cont, T, Nn, M, ragged):
    B = T * Nn
    h = N.Handle(0, N.Dims(T, Nn, D, A, int(cont), H, 4, M, 1, 0))
    L = h.layout
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    rng = np.random.default_rng(1000 + i)
    params, flat = random_params(L, names, D, A, cont, rng)
    ro, host = synth(T, Nn, D, A, cont, seed=2000 + i)
    pd = torch.from_numpy(flat).to(dev())
    outs = {k: torch.empty(B, device=dev()) for k in
            ("log_probs", "values", "next_values", "advantages", "returns")}
    lo = N.LearnOutputs(*[outs[k].data_ptr() for k in
                          ("log_probs", "values", "next_values", "advantages", "returns")])
    hp = hparams()
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), pd.data_ptr(),
                                   ctypes.byref(hp), ctypes.byref(lo), stream()))
    mb = max(B // M - ragged, 1)
    idx = np.random.RandomState(3000 + i).permutation(B)[:mb].astype(np.int32)
    idx_d = torch.from_numpy(idx).to(dev())
    g = torch.zeros(L.total, device=dev())
    loss4 = (ctypes.c_float * 4)()
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, pd.data_ptr(), idx_d.data_ptr(), mb, mb,
                                          ctypes.byref(hp), g.data_ptr(), loss4, stream()))
    torch.cuda.synchronize()
    got_flat = g.cpu().numpy()
    got = np.concatenate([got_flat[L.offset[k]:L.offset[k] + L.numel[k]] for k in range(L.count)])
    o = {k: v.cpu().numpy() for k, v in outs.items()}
    obs, _, act, *_ = host
    obs_f = obs.reshape(B, D)
    act_f = act.reshape(B, A) if cont else act.reshape(B)
    args = (obs_f[idx], act_f[idx], o["log_probs"][idx], o["advantages"][idx], o["returns"][idx])
    loss, comps, grads = P.minibatch_loss_grads(params, *args, P.Hyper(), cont, dt=np.float64)
    exact = np.concatenate([np.asarray(grads[n], np.float64).ravel() for n in names])
    scale = np.abs(exact).max()
    kernel = "sample-split" if sample_split(D, A, cont) else "two-team"
    assert np.abs(got - exact).max() <= 2e-5 * scale, (kernel, np.abs(got - exact).max() / scale)
    for k, n in enumerate(names):
        a = got[sum(L.numel[j] for j in range(k)):][:L.numel[k]]
        b = exact[sum(L.numel[j] for j in range(k)):][:L.numel[k]]
        s = max(np.abs(b).max(), 1e-3 * scale)
        assert np.abs(a - b).max() <= 1e-4 * s, (kernel, n, np.abs(a - b).max() / s)
    assert abs(loss4[0] - loss) <= 2e-5 * max(1.0, abs(loss)), (kernel, loss4[0], loss)
    assert abs(loss4[3] - comps["entropy"]) <= 2e-5 * max(1.0, abs(comps["entropy"]))
