"""GPU tests of the data-parallel learn at world size 8.

RCCL refuses two ranks on one device, so the N-rank path runs here as a single-device loopback
group (dppo_loopback_group): 8 handles, rank r owning envs [r*Nl, (r+1)*Nl) of the global batch,
driven concurrently from 8 host threads on 8 streams; every exchange RCCL would carry (advantage
(sum, sum^2) once, gradient + loss partials per minibatch) is summed on the device in rank order.
Everything else -- the kernels, the global divisors, the rank-0-only continuous entropy constant,
the shard selection of global minibatches -- is the production code path.

Two minibatch semantics (dppo_dims.global_minibatches):
* local (0, the default): each rank permutes its own samples; global minibatch j is the union of
  the ranks' local minibatches j.  Oracle: ONE learn of the global batch whose minibatch j is
  that union.
* global (1): every rank holds the reference's permutations of the GLOBAL batch (ppo.py:252-255)
  and processes its members of each global minibatch.  Oracle: the reference learn() of the
  global batch with those permutations -- i.e. world 8 must reproduce world 1.

Full BASELINE configs[4] size (CartPole, 8 x 8,192 envs = 65,536, T = 128): the 8-rank learn in
either mode against a world-1 libdppo learn of the 65,536-env buffer with the equivalent global
permutations (the oracle would need ~90 s there).
"""
import ctypes
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import diamond
from diamond import _native as N
from oracle import ppo_np as P

from gpu_helpers import H, dev, hparams, random_params, stream, synth

WORLD = 8


def shard(host, r, Nl):
    sl = slice(r * Nl, (r + 1) * Nl)
    obs, nobs, act, rew, te, tr = host
    exp = [[obs[k, sl], nobs[k, sl], act[k, sl], rew[k, sl], te[k, sl].astype(bool),
            tr[k, sl].astype(bool)] for k in range(obs.shape[0])]
    return exp


def run_loopback(T, Nl, D, A, cont, E, M, flat0, host, perms, global_mb, targets=False):
    """8 ranks in one loopback group; returns per-rank (params, trace).  targets: `perms` holds
    Fisher-Yates swap targets (dppo_learn_targets_f32: resolved on the device)."""
    handles = [N.Handle(0, N.Dims(T, Nl, D, A, int(cont), H, E, M, WORLD, r, int(global_mb)))
               for r in range(WORLD)]
    N.loopback_group(handles)
    hp = hparams()
    state = []
    for r in range(WORLD):
        ro = diamond.engine.stage_experience(shard(host, r, Nl), dev(), cont)
        state.append({"ro": ro, "st": ro.as_struct(), "p": torch.from_numpy(flat0).to(dev()),
                      "m": torch.zeros(len(flat0), device=dev()),
                      "v": torch.zeros(len(flat0), device=dev()), "rc": None, "err": b""})
    torch.cuda.synchronize()

    def run(r):
        torch.cuda.set_device(0)
        s = torch.cuda.Stream(device=dev())
        x = state[r]
        pr = perms if global_mb else perms[r]
        fn = handles[r].lib.dppo_learn_targets_f32 if targets else handles[r].lib.dppo_learn_f32
        x["rc"] = fn(handles[r].h, ctypes.byref(x["st"]), x["p"].data_ptr(), x["m"].data_ptr(),
                     x["v"].data_ptr(), ctypes.byref(hp), pr.ctypes.data, None, s.cuda_stream)
        if x["rc"] != 0:
            x["err"] = handles[r].lib.dppo_last_error()   # thread-local: read on this thread
        s.synchronize()

    th = [threading.Thread(target=run, args=(r,)) for r in range(WORLD)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    assert all(not x.is_alive() for x in th)
    bad = [(r, x["rc"], x["err"]) for r, x in enumerate(state) if x["rc"] != 0]
    assert not bad, bad
    torch.cuda.synchronize()
    out = [(x["p"].cpu().numpy(), handles[r].trace(E * M)) for r, x in enumerate(state)]
    for h in handles:
        h.close()
    return out


def run_single(T, Ng, D, A, cont, E, M, flat0, host, perms_g):
    """World-1 libdppo learn of the whole global buffer with the given global permutations."""
    h = N.Handle(0, N.Dims(T, Ng, D, A, int(cont), H, E, M, 1, 0))
    obs, nobs, act, rew, te, tr = host
    exp = [[obs[k], nobs[k], act[k], rew[k], te[k].astype(bool), tr[k].astype(bool)]
           for k in range(T)]
    ro = diamond.engine.stage_experience(exp, dev(), cont)
    p = torch.from_numpy(flat0).to(dev())
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    hp = hparams()
    pg = np.ascontiguousarray(perms_g, dtype=np.int32)
    N.check(h.lib.dppo_learn_f32(h.h, ctypes.byref(ro.as_struct()), p.data_ptr(), m.data_ptr(),
                                 v.data_ptr(), ctypes.byref(hp), pg.ctypes.data, None, stream()))
    torch.cuda.synchronize()
    res = (p.cpu().numpy(), h.trace(E * M))
    h.close()
    return res


def union_perms(perms, T, Nl, E, M):
    """Global permutations whose minibatch j is the union of the ranks' local minibatches j."""
    Ng, B = Nl * WORLD, T * Nl
    mb = B // M
    to_global = lambda r, i: (i // Nl) * Ng + r * Nl + i % Nl
    return np.stack([np.concatenate([to_global(r, perms[r][e, j * mb:(j + 1) * mb])
                                     for j in range(M) for r in range(WORLD)])
                     for e in range(E)])


def setup(T, Nl, D, A, cont, seed):
    Ng = Nl * WORLD
    L = N.param_layout(N.Dims(T, Nl, D, A, int(cont), H, 4, 8, 1, 0))
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    params, flat0 = random_params(L, names, D, A, cont, np.random.default_rng(seed))
    _, host = synth(T, Ng, D, A, cont, seed)
    host = tuple(x if x.dtype != np.uint8 else x.astype(bool) for x in host)
    return L, names, params, flat0, host


def check_vs_oracle(out, params, names, L, host, perms_g, cont, E, M):
    adam = P.new_adam_state(params, names)
    ref = P.learn(params, adam, list(host), P.Hyper(), 3e-4, cont, perms=perms_g)
    flats = [p for p, _ in out]
    for r in range(1, WORLD):
        assert np.array_equal(flats[0], flats[r])  # replicated clip + Adam on identical sums
    for r in range(WORLD):
        tr = out[r][1]
        np.testing.assert_allclose(tr[:, 0], ref["loss"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(tr[:, 4], ref["norm"], rtol=1e-4, atol=1e-5)
    for i, n in enumerate(names):
        np.testing.assert_allclose(flats[0][L.offset[i]:L.offset[i] + L.numel[i]],
                                   params[n].ravel(), rtol=0, atol=2e-5, err_msg=n)


@pytest.mark.parametrize("cont", [False, True])
def test_world8_local_minibatches_vs_oracle(cont):
    T, Nl, E, M = 16, 32, 4, 8
    D, A = (17, 6) if cont else (4, 2)
    L, names, params, flat0, host = setup(T, Nl, D, A, cont, seed=21 + cont)
    B = T * Nl
    perms = [np.stack([np.random.RandomState(100 + r).permutation(B) for _ in range(E)])
             .astype(np.int32) for r in range(WORLD)]
    out = run_loopback(T, Nl, D, A, cont, E, M, flat0, host, perms, global_mb=False)
    check_vs_oracle(out, params, names, L, host, union_perms(perms, T, Nl, E, M), cont, E, M)


@pytest.mark.parametrize("cont", [False, True])
def test_world8_global_minibatches_reproduce_world1_oracle(cont):
    """global_minibatches: the 8-rank learn IS the reference learn() of the global batch (same
    np.random.permutation draws over all T*N*8 samples)."""
    T, Nl, E, M = 16, 32, 4, 8
    D, A = (17, 6) if cont else (4, 2)
    L, names, params, flat0, host = setup(T, Nl, D, A, cont, seed=31 + cont)
    Bg = T * Nl * WORLD
    rs = np.random.RandomState(42)
    perms_g = np.stack([rs.permutation(Bg) for _ in range(E)]).astype(np.int32)
    out = run_loopback(T, Nl, D, A, cont, E, M, flat0, host, perms_g, global_mb=True)
    check_vs_oracle(out, params, names, L, host, perms_g, cont, E, M)
    # and against the single-GPU libdppo learn of the same global buffer
    single = run_single(T, Nl * WORLD, D, A, cont, E, M, flat0, host, perms_g)
    np.testing.assert_allclose(out[0][1][:, 0], single[1][:, 0], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(out[0][0], single[0], rtol=0, atol=5e-6)


def test_global_minibatch_shares_are_uneven_and_exact():
    """Small shards make the per-rank shares of a global minibatch very uneven (some zero):
    T = 4, 2 envs per rank, 8 minibatches of 8 global samples."""
    T, Nl, E, M = 4, 2, 4, 8
    D, A = 4, 3
    L, names, params, flat0, host = setup(T, Nl, D, A, False, seed=5)
    Bg = T * Nl * WORLD
    rs = np.random.RandomState(3)
    perms_g = np.stack([rs.permutation(Bg) for _ in range(E)]).astype(np.int32)
    Ng = Nl * WORLD
    counts = np.array([[[((perms_g[e, j * 8:(j + 1) * 8] % Ng) // Nl == r).sum()
                         for r in range(WORLD)] for j in range(M)] for e in range(E)])
    assert (counts == 0).any() and counts.max() >= 3
    out = run_loopback(T, Nl, D, A, False, E, M, flat0, host, perms_g, global_mb=True)
    check_vs_oracle(out, params, names, L, host, perms_g, False, E, M)


def _perms_and_targets(n, E, seed):
    key, pos, _ = N.mt_state(np.random.RandomState(seed))
    perms = np.empty(E * n, np.int32)
    N.perm_numpy(key.copy(), pos, n, E, perms)
    tg = np.empty(E * n, np.int32)
    N.perm_targets_numpy(key.copy(), pos, n, E, tg)
    return perms.reshape(E, n), tg.reshape(E, n)


@pytest.mark.parametrize("walk", ["1", "0"])
@pytest.mark.parametrize("T,Nl,A", [(16, 32, 2), (4, 2, 3)])
def test_world8_global_minibatches_from_swap_targets(monkeypatch, walk, T, Nl, A):
    """Global minibatches from the device-resolved swap targets (how the engine runs them at
    C5 sizes): with the value walk (each rank walks only its own samples to their positions,
    DPPO_PERM_WALK=1, the default) and with the whole-permutation resolution (=0), every rank's
    learn equals, bit for bit, the learn from the host-resolved permutations (the same members of
    every global minibatch, in permutation order)."""
    monkeypatch.setenv("DPPO_PERM_WALK", walk)
    E, M, D = 4, 8, 4
    L, names, params, flat0, host = setup(T, Nl, D, A, False, seed=9 + T)
    perms, tg = _perms_and_targets(T * Nl * WORLD, E, seed=77 + T)
    ref = run_loopback(T, Nl, D, A, False, E, M, flat0, host, perms, global_mb=True)
    got = run_loopback(T, Nl, D, A, False, E, M, flat0, host, tg, global_mb=True, targets=True)
    for r in range(WORLD):
        assert np.array_equal(got[r][0], ref[r][0]) and np.array_equal(got[r][1], ref[r][1]), r


@pytest.mark.parametrize("global_mb", [False, True, "targets"])
def test_world8_c5_full_size_matches_single_gpu(global_mb):
    """BASELINE configs[4]: CartPole, 8 ranks x 8,192 envs (65,536), T = 128, mb 1,048,576
    global.  The 8-rank learn against the world-1 learn of the same 65,536-env buffer with the
    equivalent global permutations: identical parameters on every rank, losses rel 2e-5,
    parameters 1e-5 abs after 32 Adam steps."""
    T, Nl, D, A, E, M = 128, 8192, 4, 2, 4, 8
    L, names, params, flat0, host = setup(T, Nl, D, A, False, seed=7)
    B = T * Nl
    targets = global_mb == "targets"   # the engine's path at this size: swap targets, walked
    if global_mb:
        perms_g, tg = _perms_and_targets(B * WORLD, E, seed=42)
        perms = tg if targets else perms_g
    else:
        perms = []
        for r in range(WORLD):
            key, pos, _ = N.mt_state(np.random.RandomState(100 + r))
            pr = np.empty(E * B, np.int32)
            N.perm_numpy(key, pos, B, E, pr)
            perms.append(pr.reshape(E, B))
        perms_g = union_perms(perms, T, Nl, E, M)
    out = run_loopback(T, Nl, D, A, False, E, M, flat0, host, perms, global_mb=bool(global_mb),
                       targets=targets)
    single = run_single(T, Nl * WORLD, D, A, False, E, M, flat0, host, perms_g)
    for r in range(1, WORLD):
        assert np.array_equal(out[0][0], out[r][0])
    np.testing.assert_allclose(out[0][1][:, 0], single[1][:, 0], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(out[0][1][:, 4], single[1][:, 4], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(out[0][0], single[0], rtol=0, atol=1e-5)
