"""The old-policy evaluation's next-value reuse (csrc/mlp.hip eval_kernel: reused next values plus the wave-run critic pass).

The reference evaluates the critic on every next_obs (ppo.py:235-238), but its rollout stores the
array env.step returned as next_obs[t] and -- unless that env was reset -- feeds the same array in
as obs[t+1] (ppo.py:163-179).  Where next_obs[i] is bitwise obs[i + N], libdppo takes V(next_obs[i])
from values[i + N] (computed by the same instructions on the same bits) and runs the critic only
on the remaining samples, compacted.  These tests hold the reuse path to bit-identity with the full
evaluation (a handle created with DPPO_EVAL_REUSE=0) on chained, unchained and partly chained
rollouts, ragged shapes and both head types."""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from diamond import _native as N

from gpu_helpers import H, dev, hparams, random_params, stream
from oracle import ppo_np as P


def _rollout(T, Nn, D, A, cont, seed, chain_frac):
    import diamond
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((T, Nn, D), dtype=np.float32)
    nobs = rng.standard_normal((T, Nn, D), dtype=np.float32)
    act = (rng.standard_normal((T, Nn, A), dtype=np.float32) if cont
           else rng.integers(0, A, (T, Nn)).astype(np.int32))
    rew = rng.normal(1.0, 1.0, (T, Nn)).astype(np.float32)
    te = (rng.random((T, Nn)) < 0.03).astype(bool)
    tr = (rng.random((T, Nn)) < 0.01).astype(bool)
    # chain a fraction of the steps: obs[t+1] = next_obs[t] (the rollout's invariant); an env
    # that terminated or truncated at t is reset instead
    chain = (rng.random((T - 1, Nn)) < chain_frac) & ~(te[:-1] | tr[:-1])
    obs[1:] = np.where(chain[:, :, None], nobs[:-1], obs[1:])
    # one near miss: equal but for the sign of zero (bitwise different -> no reuse)
    if T > 2 and Nn > 3:
        nobs[1, 3] = obs[2, 3]
        nobs[1, 3, 0] = -0.0
        obs[2, 3, 0] = 0.0
    exp = [[obs[t], nobs[t], act[t], rew[t], te[t], tr[t]] for t in range(T)]
    return diamond.engine.stage_experience(exp, dev(), cont)


def _prepare(reuse, T, Nn, D, A, cont, ro, flat):
    old = os.environ.get("DPPO_EVAL_REUSE")
    os.environ["DPPO_EVAL_REUSE"] = "1" if reuse else "0"
    try:
        h = N.Handle(0, N.Dims(T, Nn, D, A, int(cont), H, 4, 4, 1, 0))
    finally:
        if old is None:
            os.environ.pop("DPPO_EVAL_REUSE")
        else:
            os.environ["DPPO_EVAL_REUSE"] = old
    B = T * Nn
    outs = {k: torch.full((B,), float("nan"), device=dev()) for k in
            ("log_probs", "values", "next_values", "advantages", "returns")}
    lo = N.LearnOutputs(*[outs[k].data_ptr() for k in
                          ("log_probs", "values", "next_values", "advantages", "returns")])
    hp = hparams()
    pd = torch.from_numpy(flat).to(dev())
    res = []
    for _ in range(3):   # repeated launches: the ping-pong list counters reset correctly
        N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), pd.data_ptr(),
                                       ctypes.byref(hp), ctypes.byref(lo), stream()))
        torch.cuda.synchronize()
        res.append({k: v.cpu().numpy().copy() for k, v in outs.items()})
    h.close()
    return res


@pytest.mark.parametrize("T,Nn,D,A,cont,chain_frac", [
    (16, 64, 4, 2, False, 1.0),      # fully chained CartPole-shaped rollout
    (16, 64, 4, 2, False, 0.0),      # nothing to reuse: every sample in the critic pass
    (24, 40, 8, 4, False, 0.5),      # half chained, 40 envs (partial 32-sample tiles)
    (8, 33, 17, 6, True, 0.8),       # Gaussian head, 17 inputs, ragged env count
    (128, 256, 4, 2, False, 0.97),   # a longer rollout with a realistic reset rate
    (2, 5, 3, 3, False, 1.0),        # minimal T for reuse
    (8, 40, 6, 12, False, 0.5),      # 9-16 actions: the 16-head eval build
    (8, 33, 5, 10, True, 0.8),
    (1, 16, 4, 2, False, 1.0),       # T = 1: no next row, the full evaluation
])
def test_next_value_reuse_is_bit_identical(T, Nn, D, A, cont, chain_frac):
    L = N.param_layout(N.Dims(T, Nn, D, A, int(cont), H, 4, 4, 1, 0))
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    _, flat = random_params(L, names, D, A, cont, np.random.default_rng(T * Nn + D))
    ro = _rollout(T, Nn, D, A, cont, seed=T + Nn, chain_frac=chain_frac)
    full = _prepare(False, T, Nn, D, A, cont, ro, flat)
    fast = _prepare(True, T, Nn, D, A, cont, ro, flat)
    for k in full[0]:
        assert not np.isnan(full[0][k]).any(), k
        for rep in range(3):
            assert np.array_equal(full[0][k].view(np.uint32), fast[rep][k].view(np.uint32)), \
                (k, rep, int(np.sum(full[0][k] != fast[rep][k])))


@pytest.mark.parametrize("D,cont", [(8, False), (4, False), (20, True)])
def test_unaligned_observation_buffers_take_the_4b_path(D, cont):
    """The eval and pack kernels read observation rows of a multiple of 4 features with 16-B loads
    only from 16-B aligned buffers (checked on the host); the same rollout with obs / next_obs
    moved to a 4-B aligned address gives the same bits through the per-feature path."""
    T, Nn, A = 16, 48, (3 if cont else 4)
    L = N.param_layout(N.Dims(T, Nn, D, A, int(cont), H, 4, 4, 1, 0))
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    _, flat = random_params(L, names, D, A, cont, np.random.default_rng(D))
    ro = _rollout(T, Nn, D, A, cont, seed=7 + D, chain_frac=0.9)
    ref = _prepare(True, T, Nn, D, A, cont, ro, flat)
    st = ro.as_struct()
    keep = []
    for f in ("obs", "next_obs"):
        t = getattr(ro, f).reshape(-1)
        buf = torch.empty(t.numel() + 1, device=dev())
        buf[1:].copy_(t)
        assert buf[1:].data_ptr() % 16 != 0
        setattr(st, f, buf[1:].data_ptr())
        keep.append(buf)
    torch.cuda.synchronize()

    class _Shifted:
        def as_struct(self):
            return st

    got = _prepare(True, T, Nn, D, A, cont, _Shifted(), flat)
    for k in ref[0]:
        for rep in range(3):
            assert np.array_equal(ref[0][k].view(np.uint32), got[rep][k].view(np.uint32)), (k, rep)
