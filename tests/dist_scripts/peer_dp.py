"""One rank of a `world`-process job on ONE GPU whose ranks exchange through the peer exchange
(csrc/peer.hip: every rank's buffer mapped into every other rank over IPC, one-shot all-reduce),
for tests/test_gpu_peer.py.  RCCL refuses two ranks on one device, so this is how the peer path
runs on a one-GPU box; on a node the same code maps the buffers over xGMI.

kind "handle": the C ABI directly -- the exchange self-test, the latency of one gradient-sized
exchange, then dppo_learn_f32 on this rank's env shard in both minibatch modes, against the
world-1 learn of the global buffer (rank 0 runs it).  kind "agent": the drop-in PPO under
DPPO_COMM=peer (engine._init_comm maps, self-tests and agrees), one learn per rank.
Results go to `out_path` (npz).  Test infrastructure only."""
import ctypes
import os
import sys

import numpy as np


def _paths():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for p in (os.path.join(root, "diamond-ppo_amd"), root, os.path.join(root, "tests"),
              os.path.join(root, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _global_setup(T, Ng, D, A, cont, E, M, seed):
    from diamond import _native as N
    from gpu_helpers import H, random_params, synth
    from oracle import ppo_np as P
    L = N.param_layout(N.Dims(T, Ng, D, A, int(cont), H, E, M, 1, 0))
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    params, flat0 = random_params(L, names, D, A, cont, np.random.default_rng(seed))
    _, host = synth(T, Ng, D, A, cont, seed)
    host = tuple(x if x.dtype != np.uint8 else x.astype(bool) for x in host)
    return flat0, host


def _learn(h, host, lo, hi, flat0, perms, cont):
    import torch
    import diamond
    from gpu_helpers import dev, hparams, stream
    from diamond import _native as N
    obs, nobs, act, rew, te, tr = host
    exp = [[obs[k, lo:hi], nobs[k, lo:hi], act[k, lo:hi], rew[k, lo:hi], te[k, lo:hi],
            tr[k, lo:hi]] for k in range(obs.shape[0])]
    ro = diamond.engine.stage_experience(exp, dev(), cont)
    p = torch.from_numpy(flat0).to(dev())
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    hp = hparams()
    pg = np.ascontiguousarray(perms, dtype=np.int32)
    N.check(h.lib.dppo_learn_f32(h.h, ctypes.byref(ro.as_struct()), p.data_ptr(), m.data_ptr(),
                                 v.data_ptr(), ctypes.byref(hp), pg.ctypes.data, None, stream()))
    torch.cuda.synchronize()
    return p.cpu().numpy()


def run_handle(rank, world, out):
    import torch
    import torch.distributed as dist
    from diamond import _native as N
    from gpu_helpers import H, stream
    T, Nl, D, A, E, M = 16, 32, 4, 2, 4, 8
    Ng, B = Nl * world, T * Nl
    res = {}
    for gmb in (0, 1):
        h = N.Handle(0, N.Dims(T, Nl, D, A, 0, H, E, M, world, rank, gmb))
        handles = [None] * world
        dist.all_gather_object(handles, h.peer_export())
        err = h.peer_open(world, rank, b"".join(handles), shared_device=True)
        assert not err, err
        err = h.peer_selftest(stream())
        assert not err, err
        if gmb == 0:
            # latency of one gradient-sized exchange (P + 8 floats), 200 back to back
            n = h.layout.total + 8
            x = torch.zeros(n, device="cuda:0")   # stays 0 through 201 sums
            dist.barrier()
            h.peer_allreduce(x.data_ptr(), n, False, stream())
            torch.cuda.synchronize()
            dist.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(200):
                h.peer_allreduce(x.data_ptr(), n, False, stream())
            b.record()
            torch.cuda.synchronize()
            res["us_per_exchange"] = a.elapsed_time(b) * 1e3 / 200
            assert float(x.abs().max().item()) == 0.0
        flat0, host = _global_setup(T, Ng, D, A, False, E, M, seed=11)
        if gmb:
            rs = np.random.RandomState(42)
            perms = np.stack([rs.permutation(B * world) for _ in range(E)]).astype(np.int32)
            perms_g = perms
        else:
            perms_all = [np.stack([np.random.RandomState(100 + r).permutation(B)
                                   for _ in range(E)]).astype(np.int32) for r in range(world)]
            perms = perms_all[rank]
            mb = B // M
            to_g = lambda r, i: (i // Nl) * Ng + r * Nl + i % Nl
            perms_g = np.stack([np.concatenate([to_g(r, perms_all[r][e, j * mb:(j + 1) * mb])
                                                for j in range(M) for r in range(world)])
                                for e in range(E)])
        dist.barrier()
        res[f"params{gmb}"] = _learn(h, host, rank * Nl, (rank + 1) * Nl, flat0, perms, False)
        res[f"trace{gmb}"] = h.trace(E * M)
        h.close()
        if rank == 0:
            hs = N.Handle(0, N.Dims(T, Ng, D, A, 0, H, E, M, 1, 0))
            res[f"single{gmb}"] = _learn(hs, host, 0, Ng, flat0, perms_g, False)
            res[f"single_trace{gmb}"] = hs.trace(E * M)
            hs.close()
    np.savez(out, **res)


def run_agent(rank, world, out):
    import torch
    import diamond
    import bench
    from gpu_helpers import SpecEnvs
    T, Nl, D, A = 32, 64, 4, 2
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nl, verbose=False)
    agent = diamond.PPO(None, cfg, envs=SpecEnvs(D, A, False))
    L = agent._learner
    assert L.world == world and L.peer, (L.world, getattr(L, "peer", None))
    init = L.flat.flat.cpu().numpy()
    ro, _ = bench.synth_rollout(T, Nl, D, A, False, 0.02, 0.005, rank, agent.device)
    agent.learn_device(ro)
    torch.cuda.synchronize()
    np.savez(out, init=init, final=L.flat.flat.cpu().numpy(), trace=agent.learn_trace())
    L.close()


def run_share(rank, world, out):
    """Global minibatches with the swap targets drawn on the host (DPPO_PERM_DEVICE=1): the same
    four learns from the same parameters and NumPy state, first with one draw per rank
    (DPPO_PERM_SHARE=0), then with the node-shared draw (drawshare.py: rank 0 draws into shared
    memory, rank 1 uploads from it).  Eight learns at T=128 and 2,048 envs per rank: a draw of
    the 4 x 524,288 global swap targets takes milliseconds, and rank 1 sleeps before every other
    learn, so the leader's look-ahead runs ahead of the follower's uploads (the slot-hold
    protocol, drawshare.py, is what keeps it from drawing over one)."""
    import time
    import torch
    import diamond
    import bench
    from gpu_helpers import SpecEnvs
    T, Nl, D, A, n_learn = 128, 2048, 4, 2, 8
    res = {}
    init = None
    for tag, share in (("own", "0"), ("shared", "1")):
        os.environ["DPPO_PERM_SHARE"] = share
        cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nl, verbose=False,
                                global_minibatches=True)
        agent = diamond.PPO(None, cfg, envs=SpecEnvs(D, A, False))
        L = agent._learner
        assert L.global_mb and L.device_shuffle and L.lookahead
        assert (L.share is not None) == (share == "1"), L.share
        if init is None:
            init = L.flat.flat.detach().clone()
        else:
            L.flat.flat.copy_(init)
        ro, _ = bench.synth_rollout(T, Nl, D, A, False, 0.02, 0.005, rank, agent.device)
        np.random.seed(7)
        for i in range(n_learn):
            if rank == 1 and i % 2:
                time.sleep(0.05)
            agent.learn_device(ro)
        torch.cuda.synchronize()
        res[f"final_{tag}"] = L.flat.flat.cpu().numpy()
        res[f"trace_{tag}"] = agent.learn_trace()
        res[f"rng_{tag}"] = np.random.get_state()[1].copy()
        if L.share is not None:
            st = L.share.stats
            res["stats"] = np.array([st["shared"], st["own"], st["mismatch"], st["timeout"],
                                     int(L.share.leader)])
        L.close()
    np.savez(out, **res)


def run_dead(rank, world, out):
    """Rank 1 stops exchanging after the self-test (it sleeps past DPPO_PEER_TIMEOUT_S, as a
    hung or crashed peer would): rank 0's learn() must end with the peer-timeout error
    (DPPO_ECOMM -> RuntimeError) within the timeout, and refuse every later call."""
    import time
    import torch
    import diamond
    import bench
    from gpu_helpers import SpecEnvs
    T, Nl, D, A = 32, 64, 4, 2
    timeout = float(os.environ["DPPO_PEER_TIMEOUT_S"])
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nl, verbose=False)
    agent = diamond.PPO(None, cfg, envs=SpecEnvs(D, A, False))
    L = agent._learner
    assert L.world == world and L.peer
    ro, _ = bench.synth_rollout(T, Nl, D, A, False, 0.02, 0.005, rank, agent.device)
    torch.cuda.synchronize()
    err, again, elapsed = "", "", 0.0
    if rank == 0:
        t0 = time.perf_counter()
        try:
            agent.learn_device(ro)
            agent.learn_trace()          # synchronises: the sticky error surfaces here
        except RuntimeError as e:
            err = str(e)
        elapsed = time.perf_counter() - t0
        try:
            agent.learn_device(ro)
        except RuntimeError as e:
            again = str(e)
    else:
        time.sleep(timeout + 4.0)
    np.savez(out, err=err, again=again, elapsed=elapsed, timeout=timeout)
    L.close()


def run_selftest_fail(rank, world, out):
    """DPPO_PEER_SELFTEST_SKEW=1: rank 1's self-test contribution is wrong, so the sums are wrong
    on every rank; under DPPO_COMM=peer every rank's agent construction must raise."""
    import diamond
    from gpu_helpers import SpecEnvs
    err = ""
    try:
        diamond.PPO(None, diamond.PPOConfig(rollout_steps=8, num_envs=16, verbose=False),
                    envs=SpecEnvs(4, 2, False))
    except RuntimeError as e:
        err = str(e)
    np.savez(out, err=err)


def run(rank, world, port, kind, out, env=None):
    _paths()
    os.environ["LOCAL_RANK"] = "0"          # every rank on the one GPU
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"], os.environ["WORLD_SIZE"] = str(rank), str(world)
    os.environ["DPPO_COMM"] = "peer"
    os.environ["DPPO_PEER_TIMEOUT_S"] = "30"
    os.environ.update(env or {})
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        {"handle": run_handle, "agent": run_agent, "dead": run_dead, "share": run_share,
         "selftest_fail": run_selftest_fail}[kind](rank, world, out)
        dist.barrier()
    finally:
        dist.destroy_process_group()
