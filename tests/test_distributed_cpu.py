"""World-size-2 gloo tests (CPU) of the env-axis data-parallel decomposition dppo_learn_f32 uses
under RCCL, with the NumPy oracle as the compute:

* advantage statistics: each rank's (sum, sum of squares) all-reduced == the statistics of the
  whole [T, N_global] batch (reference ppo.py:243 normalises over ALL samples);
* gradient: each rank's per-sample gradient sum over its local minibatch, divided by the GLOBAL
  minibatch size and all-reduced (SUM) == the oracle gradient of the union minibatch
  (reference ppo.py:258-285: one optimizer step per minibatch);
* the replicated clip + Adam then yields identical parameters on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ppo_np as P


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params(D, A, seed=3):
    rng = np.random.default_rng(seed)
    H = 64
    shapes = {"base.0.weight": (H, D), "base.0.bias": (H,), "base.2.weight": (H, H),
              "base.2.bias": (H,), "actor_head.0.weight": (H, H), "actor_head.0.bias": (H,),
              "actor_head.2.weight": (A, H), "actor_head.2.bias": (A,),
              "critic_head.0.weight": (H, H), "critic_head.0.bias": (H,),
              "critic_head.2.weight": (1, H), "critic_head.2.bias": (1,)}
    return {n: (rng.standard_normal(s) * 0.3).astype(np.float32) for n, s in shapes.items()}


def _data(T, N, D, A, seed=11):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((T, N, D)).astype(np.float32)
    act = rng.integers(0, A, (T, N))
    rew = rng.normal(1, 1, (T, N)).astype(np.float32)
    te = rng.random((T, N)) < 0.05
    tr = rng.random((T, N)) < 0.02
    v = rng.standard_normal((T, N)).astype(np.float32)
    nv = rng.standard_normal((T, N)).astype(np.float32)
    return obs, act, rew, te, tr, v, nv


def _worker(rank, world, port, T, N, D, A, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs, act, rew, te, tr, v, nv = _data(T, N * world, D, A)
        sl = slice(rank * N, (rank + 1) * N)  # this rank's env shard
        adv = P.gae(rew[:, sl], te[:, sl], tr[:, sl], v[:, sl], nv[:, sl])
        # advantage statistics: local (sum, sumsq) -> all-reduce
        s = torch.tensor([adv.astype(np.float64).sum(), (adv.astype(np.float64) ** 2).sum()],
                         dtype=torch.float64)
        dist.all_reduce(s)
        n = T * N * world
        mean = s[0].item() / n
        std = np.sqrt((s[1].item() - s[0].item() * mean) / (n - 1))
        adv_n = (adv - np.float32(mean)) / (np.float32(std) + np.float32(1e-6))
        ret = v[:, sl] + adv
        params = _params(D, A)
        # local minibatch j of the rank-local permutation (seed + rank), global divisor
        B_loc, M = T * N, 4
        mb = B_loc // M
        perm = np.random.RandomState(42 + rank).permutation(B_loc)
        idx = perm[:mb]
        fl = lambda x: x.reshape(B_loc, *x.shape[2:])
        old_logp, _, _, _ = P.old_policy(params, obs[:, sl], act[:, sl], obs[:, sl])
        _, _, g = P.minibatch_loss_grads(params, fl(obs[:, sl])[idx], fl(act[:, sl])[idx],
                                         fl(old_logp)[idx], fl(adv_n)[idx], fl(ret)[idx],
                                         P.Hyper(), m_total=mb * world)
        flat = np.concatenate([g[k].ravel() for k in P.DISCRETE_NAMES])
        t = torch.from_numpy(flat.astype(np.float64))
        dist.all_reduce(t)
        out_q.put((rank, float(mean), float(std), t.numpy(), idx + rank * 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_global_minibatch():
    T, N, D, A, world = 8, 16, 4, 2, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, N, D, A, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, mean, std, g, idx = q.get(timeout=240)
        res[r] = (mean, std, g, idx)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # (1) statistics equal the global batch's
    obs, act, rew, te, tr, v, nv = _data(T, N * world, D, A)
    adv_g = P.gae(rew, te, tr, v, nv)
    mean_g, std_g = P.adv_stats(adv_g)
    for r in range(world):
        assert abs(res[r][0] - mean_g) < 1e-6 and abs(res[r][1] - std_g) < 1e-6
    # (2) all-reduced gradient == oracle gradient of the union minibatch
    params = _params(D, A)
    adv_n = P.normalize_adv(adv_g)
    ret = v + adv_g
    old_logp, _, _, _ = P.old_policy(params, obs, act, obs)
    rows_o, rows_a, rows_lp, rows_adv, rows_ret = [], [], [], [], []
    for r in range(world):
        sl = slice(r * N, (r + 1) * N)
        fl = lambda x: x[:, sl].reshape(T * N, *x.shape[2:])
        idx = res[r][3]
        rows_o.append(fl(obs)[idx]); rows_a.append(fl(act)[idx]); rows_lp.append(fl(old_logp)[idx])
        rows_adv.append(fl(adv_n)[idx]); rows_ret.append(fl(ret)[idx])
    cat = np.concatenate
    _, _, g = P.minibatch_loss_grads(params, cat(rows_o), cat(rows_a), cat(rows_lp),
                                     cat(rows_adv), cat(rows_ret), P.Hyper())
    ref = np.concatenate([g[k].ravel() for k in P.DISCRETE_NAMES])
    for r in range(world):
        np.testing.assert_allclose(res[r][2], ref, rtol=1e-4, atol=1e-6 * np.abs(ref).max())
    assert np.array_equal(res[0][2], res[1][2])  # identical on every rank -> replicated Adam
