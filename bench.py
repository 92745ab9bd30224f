#!/usr/bin/env python3
"""Benchmark: env-steps/s of GAE + PPO update (one learn()) on synthetic [128 x num_envs] buffers.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config lunar8192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W [--config c5]

``python bench.py --gpus N`` with N > 1 and no launcher around it starts the N ranks itself (one
child torch.distributed.run job; the parent touches no GPU) and exits with the job's status; a
launcher whose world size differs from ``--gpus`` is an error (exit 2).

A "step" is one full PPO.learn() (reference diamond/ppo.py:224-287) over one rollout buffer
already resident in HBM: old-policy eval, GAE, returns, advantage normalisation, E x M = 32
minibatch {forward, loss, backward, clip, Adam} steps and the LR-scheduler step.  The minibatch
permutations are drawn from the global NumPy RNG inside the step, bit-exactly as the reference.

Default workload (BASELINE.json configs[2]): LunarLander-shaped PPO, T = 128,
num_envs = 8192 per GPU -- the largest single-GPU configuration, and the north star's GAE size
(weak scaling: each rank owns 8192 envs, the gradient is exchanged once per minibatch), obs_dim
8, 4 actions, hidden 64, E = 4, M = 8.  ``--config c5`` is BASELINE configs[4] as a
STRONG-scaling run: 65,536 envs in total split over the ranks (8,192 per GPU at 8); its
``update_steps_per_s`` (minibatch optimizer steps per second) is the quantity the north star's
>= 6x-at-8-GPUs target is stated in.  Synthetic data: obs/next_obs ~ N(0,1), rewards ~ N(1,1),
term ~ Bern(0.02), trunc ~ Bern(0.005), uniform actions, default_rng(rank); random-init weights
of the reference architecture.

Rank 0 prints ONE JSON line.  ``value`` comes from a timed pass with nothing but the learn()
work in the stream.  A second timed pass of the same K learns stamps every kernel with its own
start/end HIP events (libdppo timing mode): ``kernels``, ``device_ms_per_step`` and ``roofline``
(the dominant kernel by device time, its average launch duration, algorithmic FLOP per launch)
come from it, never the throughput.  At N = 1 the line also carries ``configs_extra`` (C2
CartPole 4096, C4 HalfCheetah 4096 and C5's 65,536 envs on one GPU -- the strong-scaling
anchor), ``roofline_gae`` (the GAE kernel at num_envs = 8192 over 16 rotating buffer sets, 368 MB
> the 256 MB Infinity Cache; ``roofline_gae_affine`` the tolerance-mode kernel, and
``roofline_gae_65536`` both at C5's one-GPU 65,536 envs) and ``cpu_baseline``: the PyTorch-CPU
restatement of the reference path (oracle/ppo_torch.py) timed for one full learn() of the
headline workload on the host cores, with the NumPy oracle beside it as ``cpu_baseline_numpy``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
# DPPO_PY_ROOT (A/B timing only): import the diamond package from another tree
sys.path.insert(0, os.environ.get("DPPO_PY_ROOT") or os.path.join(ROOT, "diamond-ppo_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy 6290
FP32_PEAK_TFLOPS = 157.3    # MI355X fp32 MFMA (= vector) dense peak
H = 64

CONFIGS = {
    # name: (model, T, N, D, A, continuous, p_term, p_trunc, scaling)
    #   scaling "weak": N envs per GPU; "strong": N envs in total, split over the ranks
    "cartpole4096": ("CartPole-v1 PPO", 128, 4096, 4, 2, False, 0.02, 0.005, "weak"),
    "lunar8192": ("LunarLander-v3 PPO", 128, 8192, 8, 4, False, 0.02, 0.005, "weak"),
    "cheetah4096": ("HalfCheetah-v5 ContinuousPPO", 128, 4096, 17, 6, True, 0.0, 0.001, "weak"),
    "cartpole8192": ("CartPole-shaped PPO (8,192 envs/GPU: configs[4] shard)", 128, 8192, 4, 2,
                     False, 0.02, 0.005, "weak"),
    # BASELINE configs[4]: 65,536 CartPole-shaped envs in total (8,192 per GPU at 8 GPUs)
    "c5": ("CartPole-shaped PPO, 65,536 envs in total (configs[4])", 128, 65536, 4, 2, False,
           0.02, 0.005, "strong"),
}


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


class Discrete:
    def __init__(self, n):
        self.n = int(n)


class SpecEnvs:
    """Only the spaces: learn() on staged buffers never steps an environment."""

    def __init__(self, D, A, continuous):
        self.single_observation_space = Box((D,))
        self.single_action_space = Box((A,)) if continuous else Discrete(A)


def flops_per_sample(D, A):
    """fwd MACs F = D*H + 3H^2 + H(A+1); value-only V = D*H + 2H^2 + H;
    minibatch fwd+bwd = 3F - D*H MACs."""
    F = D * H + 3 * H * H + H * (A + 1)
    V = D * H + 2 * H * H + H
    return 2 * F, 2 * V, 2 * (3 * F - D * H)


def synth_rollout(T, N, D, A, continuous, p_term, p_trunc, seed, device, chained=True):
    """A synthetic [T, N] rollout.  chained (default): the reference rollout's invariant
    (ppo.py:163-179) -- obs[t+1] is the array env.step returned as next_obs[t], except for the envs
    that terminated or truncated at t, which were reset to a fresh observation.  chained=False:
    obs and next_obs drawn independently (no step continues another)."""
    from diamond.engine import DeviceRollout
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((T, N, D), dtype=np.float32)
    nobs = rng.standard_normal((T, N, D), dtype=np.float32)
    if continuous:
        act = rng.standard_normal((T, N, A), dtype=np.float32)
    else:
        act = rng.integers(0, A, (T, N)).astype(np.int32)
    rew = rng.normal(1.0, 1.0, (T, N)).astype(np.float32)
    te = (rng.random((T, N)) < p_term).astype(np.uint8)
    tr = (rng.random((T, N)) < p_trunc).astype(np.uint8)
    if chained:
        done = (te | tr).astype(bool)
        obs[1:] = np.where(done[:-1, :, None], obs[1:], nobs[:-1])
    g = lambda x: torch.from_numpy(x).to(device)
    return DeviceRollout(g(obs), g(nobs), g(act), g(rew), g(te), g(tr)), (obs, nobs, act, rew, te, tr)


def gae_roofline(device, T=128, N=8192, sets=None, reps=4, mode=0):
    """GAE kernel alone over distinct buffer sets rotated past the 256 MB Infinity Cache (at
    N = 8192: 16 sets x 22 B/elem x 1,048,576 elem = 369 MB; at N = 65,536: 2 sets x 184 MB),
    launched back to back; each launch's duration comes from the HIP event pair libdppo attaches
    to the kernel itself (timing mode, hipExtLaunchKernel).  mode: 0 = the bit-exact serial scan
    (the default), 1 = the chunked affine scan (tolerance mode, dppo_set_gae_mode)."""
    from diamond import _native as NN
    if sets is None:
        sets = max(2, -(-369 * 2 ** 20 // (22 * T * N)))
    if N >= 65536:
        reps = max(reps, 16)
    h = NN.Handle(device.index or 0, NN.Dims(T, N, 1, 1, 0, 64, 1, 1, 1, 0))
    h.set_gae_mode(mode)
    rng = np.random.default_rng(1)
    bufs = []
    for _ in range(sets):
        bufs.append([torch.from_numpy(rng.normal(1, 1, (T, N)).astype(np.float32)).to(device),
                     torch.from_numpy((rng.random((T, N)) < 0.02).astype(np.uint8)).to(device),
                     torch.from_numpy((rng.random((T, N)) < 0.005).astype(np.uint8)).to(device),
                     torch.from_numpy(rng.standard_normal((T, N), dtype=np.float32)).to(device),
                     torch.from_numpy(rng.standard_normal((T, N), dtype=np.float32)).to(device),
                     torch.empty(T, N, device=device), torch.empty(T, N, device=device)])
    s = torch.cuda.current_stream(device)

    def launch(b):
        NN.check(h.lib.dppo_gae_f32(h.h, *[x.data_ptr() for x in b], 0.99, 0.95, s.cuda_stream))

    def probe(b):  # the same bytes, no recurrence (dppo_gae_stream_probe): the launch's ceiling
        NN.check(h.lib.dppo_gae_stream_probe(h.h, *[x.data_ptr() for x in b], s.cuda_stream),
                 "dppo_gae_stream_probe")

    for b in bufs:
        launch(b)
        probe(b)
    torch.cuda.synchronize(device)
    h.set_timing(True)
    for _ in range(reps):  # alternating rounds over the same rotating sets
        for b in bufs:
            launch(b)
        for b in bufs:
            probe(b)
    tm = h.timing()
    ms, cnt = tm["gae"]
    pms, pcnt = tm["gae_probe"]
    h.set_timing(False)
    per = ms / cnt
    nbytes = 22 * T * N
    achieved = nbytes / (per * 1e-3) / 1e9
    ceil_us = pms / pcnt * 1e3
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = f"gae{N}" + ("_affine" if mode else "")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(key, {}).get("gae")
        except Exception:
            traffic = None
    h.close()
    del bufs
    torch.cuda.empty_cache()
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": ("gae_aff_kernel<%d>" if mode else "gae_pipe_kernel<%d>") % _gae_tile(N),
            "mode": "affine (<= 1e-6 of scale)" if mode else "exact (bit-exact serial)",
            "num_envs": N, "rollout_steps": T,
            "bytes_per_launch": nbytes, "us_per_launch": round(per * 1e3, 2),
            "launches": cnt, "rotating_sets": sets,
            # the same bytes with no recurrence (dppo_gae_stream_probe), timed in the same run
            # over the same sets: what one launch of these bytes streams at on this part
            "ceiling_us": round(ceil_us, 2),
            "ceiling_GBps": round(nbytes / (ceil_us * 1e-6) / 1e9, 1),
            "frac_of_ceiling": round(ceil_us / (per * 1e3), 4)}


def _gae_tile(N):
    """The env-tile width gae.hip's launcher picks for N (64 / 32 / 16 envs per workgroup)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if N % 64 == 0 and N // 64 >= cus:
        return 64
    return 32 if N % 32 == 0 and N // 32 >= cus else 16


def _baseline_inputs(cfg_name, seed=0):
    sys.path.insert(0, ROOT)
    from oracle import ppo_np as P
    _, T, N, D, A, cont, pt, ptr, _ = CONFIGS[cfg_name]
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((T, N, D), dtype=np.float32)
    nobs = rng.standard_normal((T, N, D), dtype=np.float32)
    act = rng.standard_normal((T, N, A), dtype=np.float32) if cont else rng.integers(0, A, (T, N))
    rew = rng.normal(1, 1, (T, N)).astype(np.float32)
    te = rng.random((T, N)) < pt
    tr = rng.random((T, N)) < ptr
    prng = np.random.default_rng(42)
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    head = "actor_mean_head" if cont else "actor_head"
    shapes = {"base.0.weight": (H, D), "base.2.weight": (H, H), f"{head}.0.weight": (H, H),
              f"{head}.2.weight": (A, H), "critic_head.0.weight": (H, H),
              "critic_head.2.weight": (1, H)}
    params = {}
    for n in names:
        if n == "actor_log_std":
            params[n] = np.zeros((1, A), np.float32)
        elif n in shapes:
            params[n] = (prng.standard_normal(shapes[n]) / np.sqrt(shapes[n][1])).astype(np.float32)
        else:
            params[n] = np.zeros(shapes[n.replace("bias", "weight")][0], np.float32)
    return (obs, nobs, act, rew, te, tr), params, names, cont, T * N


def host_cpus():
    """(CPUs the process may run on, CPUs its cgroup quota pays for or None, threads to use).
    On the GPU box the affinity mask holds the whole machine (256) while the cgroup quota is the
    box's share (16): more threads than the quota only get throttled."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return aff, quota, min(aff, quota) if quota else aff


CPU_VS_REF = "r06_cpu_baseline_vs_reference.json"


def cpu_baselines(cfg_name):
    """One full learn() of the same workload on the host cores: the PyTorch-CPU restatement
    (oracle/ppo_torch.py: the reference's own arithmetic -- autograd, torch.distributions,
    clip_grad_norm_, CPU Adam) and the NumPy oracle.  Runs in a child process that never touches
    the GPU (see cpu_baselines_child), on every CPU the process may use."""
    from oracle import ppo_np as P
    from oracle import ppo_torch as PT
    exp, params, names, cont, B = _baseline_inputs(cfg_name)
    model = PT.cpu_model()
    aff, quota, threads = host_cpus()
    torch.set_num_threads(threads)
    p1 = {k: v.copy() for k, v in params.items()}
    torch.optim.Adam([torch.zeros(1, requires_grad=True)])  # first-use imports outside the clock
    t0 = time.perf_counter()
    PT.learn(p1, exp, P.Hyper(), 3e-4, cont, rng=np.random.RandomState(42))
    dt_t = time.perf_counter() - t0
    torch_b = {"value": round(B / dt_t, 1), "unit": "env-steps/s", "cores": int(threads),
               "kind": "port", "cpu": model, "affinity_cpus": aff, "cgroup_cpus": quota,
               "process": "child started before any GPU call (no HIP runtime, no draw threads)",
               "sample": f"one full learn() of {cfg_name} (T x N = {B} samples: old-policy eval, "
                         f"GAE, 4x8 minibatch autograd/clip/Adam steps) by the PyTorch-CPU "
                         f"restatement of the reference path (oracle/ppo_torch.py), {dt_t:.2f} s "
                         f"on {threads} torch threads",
               "seconds": round(dt_t, 3)}
    try:
        from threadpoolctl import threadpool_info
        np_threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        np_threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    p2 = {k: v.copy() for k, v in params.items()}
    t0 = time.perf_counter()
    P.learn(p2, P.new_adam_state(p2, names), exp, P.Hyper(), 3e-4, cont,
            rng=np.random.RandomState(42))
    dt_n = time.perf_counter() - t0
    numpy_b = {"value": round(B / dt_n, 1), "unit": "env-steps/s", "cores": int(np_threads),
               "kind": "port", "cpu": model,
               "sample": f"the same learn() by the NumPy float32 oracle (oracle/ppo_np.py), "
                         f"{dt_n:.2f} s", "seconds": round(dt_n, 3)}
    return torch_b, numpy_b


def cpu_baselines_child(cfg_name):
    """Time cpu_baselines in a fresh interpreter started before this process makes any GPU call:
    the baseline is then not slowed by the HIP runtime's threads or the permutation pools."""
    import subprocess
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", cfg_name],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline child failed: {r.stderr[-2000:]}")
    tb, nb = json.loads(r.stdout.strip().splitlines()[-1])
    return tb, nb


def run_config(name, world, rank, dist, device, steps, warmup, kernel_timing=True,
               global_mb=False, keep_agent=False):
    """Time `steps` learn() calls of CONFIGS[name] on this rank; returns the measurement dict
    (max wall time over ranks)."""
    import diamond
    from diamond import _native as NN
    model, T, Nc, D, A, cont, pt, ptr, scaling = CONFIGS[name]
    N = Nc // world if scaling == "strong" else Nc
    if scaling == "strong" and Nc % world:
        raise SystemExit(f"{name}: {Nc} global envs do not split over {world} ranks")
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=N, verbose=False, total_steps=10 ** 12,
              global_minibatches=global_mb)
    agent = Agent(None, cfg, envs=SpecEnvs(D, A, cont))
    assert agent._learner.fused, "benchmark must exercise the fused HIP path"
    ro, _ = synth_rollout(T, N, D, A, cont, pt, ptr, seed=rank, device=device)
    torch.cuda.synchronize(device)
    for _ in range(warmup):
        agent.learn_device(ro)
    torch.cuda.synchronize(device)
    h = agent._learner.handle
    hs = agent._learner.host_seconds

    def timed_pass(instrument: bool):
        """K learns between barrier + synchronize brackets; max wall time over ranks."""
        h.set_timing(instrument)
        for k in ("perms", "enqueue", "draft_start", "draw", "slot_wait"):
            hs[k] = 0.0
        hs["calls"] = 0
        hs["lookahead_hits"] = 0
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(steps):
            agent.learn_device(ro)
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64,
                             device=device if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # Pass A (the reported throughput): no per-launch events in the stream.
    elapsed = timed_pass(False)
    host = {k: round(hs[k] / max(hs["calls"], 1) * 1e3, 4) for k in ("perms", "enqueue",
                                                                      "draft_start", "draw",
                                                                      "slot_wait")}
    hits = hs["lookahead_hits"]
    # Pass A' (reported beside it): the same learns on a rollout whose next_obs never continues
    # into obs -- the old-policy evaluation's next-value reuse (mlp.hip) then finds nothing to
    # reuse and runs the full critic pass on next_obs
    ro_chained = ro
    ro, _ = synth_rollout(T, N, D, A, cont, pt, ptr, seed=rank, device=device, chained=False)
    agent.learn_device(ro)
    elapsed_unchained = timed_pass(False)
    ro = ro_chained
    # Pass B (the per-kernel table and the roofline): the same K learns with the kernels' own
    # start/end HIP events (libdppo timing mode); never the throughput.
    timing = {k: (0.0, 0) for k in NN.TIMING_CLASSES}
    elapsed_instr = None
    if kernel_timing:
        elapsed_instr = timed_pass(True)
        timing = h.timing()
    h.set_timing(False)
    loss_trace = agent.learn_trace()
    E, M = cfg.num_epochs, cfg.num_minibatches
    B_global = T * N * world
    dom = max(timing, key=lambda k: timing[k][0])
    f_eval_full, f_eval_v, f_mb = flops_per_sample(D, A)
    mb = T * N // M
    algo = {  # (bound, algorithmic units per launch, unit)
        "grad": ("mfma", f_mb * mb, "TFLOP/s"),
        "eval": ("mfma", (f_eval_full + f_eval_v) * T * N, "TFLOP/s"),
        "gae": ("hbm", 22 * T * N, "GB/s"),
    }
    roofline = None
    if dom in algo and timing[dom][1] > 0:
        bound, units, unit = algo[dom]
        tot_ms, cnt = timing[dom]
        per_s = tot_ms / cnt * 1e-3
        if unit == "TFLOP/s":
            ach, peak = units / per_s / 1e12, FP32_PEAK_TFLOPS
        else:
            ach, peak = units / per_s / 1e9, HBM_PEAK_GBS
        roofline = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                    "frac": round(ach / peak, 4), "traffic": None, "kernel": dom,
                    "per_launch": units, "us_per_launch": round(tot_ms / cnt * 1e3, 2)}
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                tr = json.load(open(pmc)).get(name, {}).get(dom)
                if tr is not None:
                    roofline["traffic"] = tr
            except Exception:
                pass
    kernel_ms = {k: {"ms_total": round(v[0], 3), "launches": v[1],
                     "us_avg": round(v[0] / v[1] * 1e3, 2) if v[1] else 0.0}
                 for k, v in timing.items() if v[1]}
    dev_ms = sum(v[0] for v in timing.values())
    res = {
        "value": round(B_global * steps / elapsed, 1),
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "update_steps_per_s": round(E * M * steps / elapsed, 1),
        "value_unchained_obs": round(B_global * steps / elapsed_unchained, 1),
        "scaling": scaling,
        "config": {"workload": f"{model}: learn() = old-policy eval + GAE + adv-norm + "
                               f"{E}x{M} minibatch Adam steps", "name": name,
                   "baseline_config": BASELINE_INDEX.get(name),
                   "rollout_steps": T, "num_envs_per_gpu": N, "num_envs_total": N * world,
                   "obs_dim": D, "act_dim": A, "continuous": cont, "hidden": H,
                   "batch_per_learn": B_global, "minibatch": B_global // M,
                   "parallelism": f"env-axis dp{world}",
                   # the per-minibatch gradient exchange: the one-shot peer all-reduce over the
                   # ranks' xGMI-mapped buffers, or RCCL (DPPO_COMM, engine._init_comm)
                   "exchange": ("peer" if getattr(agent._learner, "peer", False) else "rccl")
                               if world > 1 else "none",
                   "minibatches": "global" if (global_mb and world > 1) else
                                  ("local-union" if world > 1 else "reference")},
        "roofline": roofline,
        "kernels": kernel_ms,
        "device_ms_per_step": round(dev_ms / steps, 4),
        "instrumented_ms_per_step": (round(elapsed_instr / steps * 1e3, 4)
                                     if elapsed_instr else None),
        "host_ms_per_step": host,
        # where the host's permutation draws ran (csrc/perm.cpp: the least busy L3 domain at first
        # use, re-chosen when draws turn slow -- engine._watch_draw)
        "host_placement": dict(getattr(NN, "perm_domain", dict)(),  # (absent: an A/B tree)
                               repin_requests=getattr(agent._learner, "repin_requests", None)),
        # the host's own work per learn (draws on the draft thread + the launching thread's
        # calls), excluding time spent blocked on the device
        "host_work_ms_per_step": round(host["draw"] + host["enqueue"] + host["draft_start"]
                                       - host["slot_wait"], 4),
        "perm_lookahead_hits": hits,
        "final_loss": float(loss_trace[-1, 0]),
    }
    if keep_agent:
        res["_agent"] = agent
    del agent, ro
    torch.cuda.synchronize(device)
    torch.cuda.empty_cache()
    return res


def exchange_report(agent, dist, device, reps=200):
    """The per-minibatch gradient exchange of a data-parallel learner: the transport engine
    selected (peer exchange over the ranks' xGMI-mapped buffers, or RCCL), its start-up
    self-test, the exchange buffer's memory type, and microseconds per gradient-sized exchange
    (P + 8 floats, `reps` back to back on the launch stream, HIP events; max over ranks)."""
    L = agent._learner
    h = L.handle
    n = h.layout.total + 8
    buf = torch.zeros(n, dtype=torch.float32, device=device)
    s = torch.cuda.current_stream(device)
    peer = bool(getattr(L, "peer", False))
    if peer:
        f = lambda: h.peer_allreduce(buf.data_ptr(), n, False, s.cuda_stream)
    else:
        f = lambda: dist.all_reduce(buf)
    for _ in range(10):
        f()
    torch.cuda.synchronize(device)
    dist.barrier()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        f()
    b.record(s)
    b.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    t = torch.tensor([us], dtype=torch.float64,
                     device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    info = h.peer_info() if peer else {}
    return {"transport": "peer" if peer else "rccl",
            "peer_selftest": getattr(L, "peer_status", "not run"),
            "memory": info.get("memory"), "fused_in_optimizer_step": info.get("fused"),
            "bytes_per_exchange": 4 * n, "us_per_exchange_max_over_ranks": round(float(t.item()), 2),
            "exchanges_timed": reps}


def multi_gpu_report(world, rank, dist, device, steps, warmup):
    """At N > 1, after the headline line's weak-scaling workload: BASELINE configs[4] as a
    STRONG-scaling run (65,536 envs split over the ranks) in both minibatch modes -- local-union
    (each rank permutes its own samples) and global (the reference's permutations of the whole
    batch, ppo.py:252-255, reproduced on every rank) -- with update-steps/s (the north star's
    >= 6x quantity) against a world-1 anchor measured on rank 0's GPU in the same job, and the
    exchange transport with its self-test outcome and latency."""
    from diamond import engine as EN
    keys = ("value", "update_steps_per_s", "ms_per_step", "device_ms_per_step",
            "host_work_ms_per_step", "host_ms_per_step")
    rep = {}
    for gmb in (False, True):
        r = run_config("c5", world, rank, dist, device, steps, warmup, global_mb=gmb,
                       keep_agent=True)
        agent = r.pop("_agent")
        row = {k: r[k] for k in keys}
        row["num_envs_per_gpu"] = r["config"]["num_envs_per_gpu"]
        row["minibatches"] = r["config"]["minibatches"]
        perm = r["kernels"].get("perm")
        row["perm_device_ms_per_step"] = round(perm["ms_total"] / steps, 4) if perm else 0.0
        if not gmb:
            rep["exchange"] = exchange_report(agent, dist, device)
        else:
            # the node-shared draw (drawshare.py): per rank {shared, own, mismatch, timeout} --
            # followers that took every draft from the leader drew nothing themselves
            sh = agent._learner.share
            mine = dict(sh.stats, leader=bool(sh.leader)) if sh is not None else None
            allst = [None] * world
            dist.all_gather_object(allst, mine)
            row["perm_share"] = allst
        rep["c5_strong_" + ("global" if gmb else "local")] = row
        del agent
        torch.cuda.empty_cache()
    anchor = None
    if rank == 0:  # the same learn on ONE GPU (the other ranks wait)
        with EN.solo():
            r1 = run_config("c5", 1, 0, None, device, steps, warmup, kernel_timing=False)
        anchor = {k: r1[k] for k in ("update_steps_per_s", "value", "ms_per_step")}
    dist.barrier()
    if anchor is not None:
        rep["c5_world1_anchor"] = anchor
        rep["c5_update_steps_speedup_vs_world1"] = {
            m: round(rep[f"c5_strong_{m}"]["update_steps_per_s"] / anchor["update_steps_per_s"], 3)
            for m in ("local", "global")}
    return rep


def spawn_ranks(n: int) -> int:
    """``python bench.py --gpus N`` (N > 1) without a torch.distributed launcher around it: start
    the N ranks as ONE child ``torch.distributed.run`` job (the parent makes no GPU call, so no
    exec-after-GPU-init and no device context in the parent) and relay its exit status; rank 0's
    JSON line reaches stdout through the inherited descriptors."""
    import socket
    import subprocess
    rehearse = os.environ.get("DPPO_BENCH_REHEARSE") == "1"
    have = torch.cuda.device_count()    # counts devices without initialising HIP (this image)
    if not rehearse and have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible (DPPO_BENCH_REHEARSE=1 "
              f"rehearses N ranks on one GPU)", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


# bench config name -> its entry in BASELINE.json "configs"
BASELINE_INDEX = {"cartpole4096": "configs[1]", "lunar8192": "configs[2]",
                  "cheetah4096": "configs[3]", "c5": "configs[4]"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); without a torch.distributed launcher, N > 1 "
                         "starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="lunar8192", choices=sorted(CONFIGS),
                    help="default: BASELINE configs[2], LunarLander N = 8192 per GPU -- the "
                         "largest single-GPU config (the north star's GAE size)")
    ap.add_argument("--global-minibatches", action="store_true",
                    help="N > 1: every rank processes its members of the reference's global "
                         "minibatches (cfg.global_minibatches) instead of local-union minibatches")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gae-roofline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="N = 1: skip the other BASELINE configs (C2, C4, C5 on one GPU); N > 1: "
                         "skip the multi_gpu legs (C5 strong scaling, both minibatch modes, "
                         "world-1 anchor, exchange latency)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no per-kernel HIP events in the timed region (no roofline)")
    ap.add_argument("--cpu-baseline-child", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_child:  # the baseline child: CPU only, prints one JSON line
        sys.path.insert(0, ROOT)
        print(json.dumps(cpu_baselines(args.cpu_baseline_child)), flush=True)
        return

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)",
              file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # first, before this process touches the GPU: the CPU path on the headline workload
        # itself (c5's 65,536 envs: its 4,096-env shape)
        baseline = cpu_baselines_child(args.config if args.config != "c5" else "cartpole4096")
    # DPPO_BENCH_REHEARSE=1: rehearse the N > 1 path on a one-GPU box -- every rank on GPU 0, a
    # gloo process group, the peer exchange between the ranks (RCCL refuses two ranks on one
    # device).  The numbers then measure ranks sharing one GPU, not scaling.
    rehearse = world > 1 and os.environ.get("DPPO_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
        os.environ["LOCAL_RANK"] = "0"   # the agents pick their device from LOCAL_RANK
        os.environ["DPPO_COMM"] = "peer"
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    main_res = run_config(args.config, world, rank, dist, device, args.steps, args.warmup,
                          kernel_timing=not args.no_kernel_timing,
                          global_mb=args.global_minibatches)
    out = None
    if rank == 0:
        out = {
            "metric": "env-steps/sec (GAE+update) on synthetic [128 x num_envs] buffers",
            "value": main_res["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": main_res["scaling"],
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "data_note": "random observations/rewards/dones in the reference rollout's layout: "
                         "obs[t+1] is next_obs[t] unless that env was reset (ppo.py:163-179); "
                         "value_unchained_obs: the same learns with independent next_obs",
        }
        out.update({k: v for k, v in main_res.items() if k not in out})
        out["device"] = {"name": torch.cuda.get_device_name(device),
                         "arch": getattr(torch.cuda.get_device_properties(device), "gcnArchName", ""),
                         "compute_units": torch.cuda.get_device_properties(device).multi_processor_count}
    if world > 1 and not args.no_extra:
        mg = multi_gpu_report(world, rank, dist, device, min(args.steps, 10), 2)
        if rank == 0:
            out["multi_gpu"] = mg
    if world == 1 and not args.no_extra:
        # the other BASELINE configs on this GPU (C3, C4), and C5's 65,536 global envs on ONE
        # GPU: the anchor of the configs[4] strong-scaling curve (`--config c5 --gpus N`)
        extra = {}
        for name in ("cartpole4096", "lunar8192", "cheetah4096", "c5"):
            if name == args.config:
                continue
            r = run_config(name, 1, 0, None, device, min(args.steps, 10), 2)
            extra[name] = {k: r[k] for k in ("value", "ms_per_step", "update_steps_per_s",
                                             "device_ms_per_step", "host_ms_per_step",
                                             "host_work_ms_per_step")}
            extra[name]["roofline"] = r["roofline"]
            extra[name]["config"] = r["config"]
        out["configs_extra"] = extra
    if rank == 0 and world == 1:
        # The headline workload moved in round 4 from configs[1] (CartPole, 4,096 envs; rounds
        # 1-3) to configs[2] (LunarLander, 8,192 envs: the largest one-GPU config and the north
        # star's GAE size); lines of different rounds compare by this key, and the configs[1]
        # number stays beside it (configs_extra.cartpole4096)
        c1 = out.get("configs_extra", {}).get("cartpole4096", {}).get("value")
        if args.config == "cartpole4096":
            c1 = out["value"]
        out["headline"] = {"name": args.config, "baseline_config": BASELINE_INDEX.get(args.config),
                           "since": "round 4 (rounds 1-3: configs[1] cartpole4096)",
                           "configs1_cartpole4096_value": c1}
    if rank == 0 and world == 1 and not args.no_gae_roofline:
        out["roofline_gae"] = gae_roofline(device)
        out["roofline_gae_affine"] = gae_roofline(device, mode=1)
        # C5's one-GPU buffer (65,536 envs, 184 MB per launch): the launch ramp amortised
        out["roofline_gae_65536"] = {"exact": gae_roofline(device, N=65536),
                                     "affine": gae_roofline(device, N=65536, mode=1)}
    if baseline is not None:
        tb, nb = baseline
        # the restatement's time over the reference's own on the same learn(), measured in the
        # build container where the reference is importable (tools/cpu_baseline_vs_reference.py;
        # the reference never travels to this box): the factor converts the port's rate into
        # an estimate of the reference path's rate on these cores
        try:
            with open(os.path.join(ROOT, "profiles", CPU_VS_REF)) as f:
                cal = json.load(f)
            r = float(cal.get("restatement_over_reference_time_median",
                              cal["restatement_over_reference_time"]))
            tb["restatement_over_reference"] = round(r, 3)
            tb["restatement_over_reference_source"] = f"profiles/{CPU_VS_REF} ({cal['cpu']}, " \
                                                      f"{cal['torch_threads']} threads, " \
                                                      f"T={cal['T']} N={cal['N']})"
            tb["reference_equivalent_value"] = round(tb["value"] * r, 1)
        except (OSError, KeyError, ValueError):
            pass
        out["cpu_baseline"] = tb
        out["cpu_baseline_numpy"] = nb
        out["speedup_vs_cpu_baseline"] = round(out["value"] / tb["value"], 1)
        if "reference_equivalent_value" in tb:
            out["speedup_vs_reference_equivalent"] = round(
                out["value"] / tb["reference_equivalent_value"], 1)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
