#!/usr/bin/env python3
"""Benchmark: env-steps/s of GAE + PPO update (one learn()) on synthetic [128 x num_envs] buffers.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cartpole4096]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one full PPO.learn() (reference diamond/ppo.py:224-287) over one rollout buffer
already resident in HBM: old-policy eval, GAE, returns, advantage normalisation, E x M = 32
minibatch {forward, loss, backward, clip, Adam} steps and the LR-scheduler step.  The minibatch
permutations are drawn from the global NumPy RNG inside the step, bit-exactly as the reference.

Workload (BASELINE.json configs[1]): CartPole-shaped PPO, T = 128,
num_envs = 4096 per GPU (weak scaling across GPUs: each rank owns 4096 envs, the gradient is
all-reduced over RCCL once per minibatch), obs_dim 4, 2 actions, hidden 64, E = 4, M = 8.
Synthetic data: obs/next_obs ~ N(0,1), rewards ~ N(1,1), term ~ Bern(0.02), trunc ~ Bern(0.005),
uniform actions, default_rng(rank); random-init weights of the reference architecture.

Rank 0 prints ONE JSON line.  ``value`` comes from a timed pass with nothing but the learn()
work in the stream.  A second timed pass of the same K learns records a HIP event pair on the
launch stream around every kernel (libdppo timing mode): it yields ``kernels``,
``device_ms_per_step`` and ``roofline`` -- the dominant kernel (largest share of device time),
its average launch duration from those events -- and its own ``instrumented_ms_per_step`` (the
event markers cost stream time, so that pass is never the throughput); ``roofline_gae`` is the GAE kernel at num_envs = 8192
over 16 rotating buffer sets (368 MB > the 256 MB Infinity Cache).  ``cpu_baseline`` is the
NumPy oracle (oracle/ppo_np.py) running one full learn() of the same workload on the host.
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
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy 6290
FP32_PEAK_TFLOPS = 157.3    # MI355X fp32 MFMA (= vector) dense peak
H = 64

CONFIGS = {
    # name: (model, T, N per GPU, D, A, continuous, p_term, p_trunc)
    "cartpole4096": ("CartPole-v1 PPO", 128, 4096, 4, 2, False, 0.02, 0.005),
    "lunar8192": ("LunarLander-v3 PPO", 128, 8192, 8, 4, False, 0.02, 0.005),
    "cheetah4096": ("HalfCheetah-v5 ContinuousPPO", 128, 4096, 17, 6, True, 0.0, 0.001),
    "cartpole8192": ("CartPole-shaped PPO (8,192 envs/GPU: configs[4] shard)", 128, 8192, 4, 2,
                     False, 0.02, 0.005),
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


def synth_rollout(T, N, D, A, continuous, p_term, p_trunc, seed, device):
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
    g = lambda x: torch.from_numpy(x).to(device)
    return DeviceRollout(g(obs), g(nobs), g(act), g(rew), g(te), g(tr)), (obs, nobs, act, rew, te, tr)


def gae_roofline(device, T=128, N=8192, sets=16, reps=4):
    """GAE kernel alone over `sets` distinct buffer sets (22 B/elem x 1,048,576 elem x 16 = 369 MB
    > 256 MB Infinity Cache), launched back to back; each launch's duration comes from the HIP
    event pair libdppo attaches to the kernel itself (timing mode, hipExtLaunchKernel)."""
    from diamond import _native as NN
    h = NN.Handle(device.index or 0, NN.Dims(T, N, 1, 1, 0, 64, 1, 1, 1, 0))
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

    for b in bufs:
        launch(b)
    torch.cuda.synchronize(device)
    h.set_timing(True)
    for _ in range(reps):
        for b in bufs:
            launch(b)
    ms, cnt = h.timing()["gae"]
    h.set_timing(False)
    per = ms / cnt
    nbytes = 22 * T * N
    achieved = nbytes / (per * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(f"gae{N}", {}).get("gae")
        except Exception:
            traffic = None
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "gae_pipe_kernel<32>", "num_envs": N, "rollout_steps": T,
            "bytes_per_launch": nbytes, "us_per_launch": round(per * 1e3, 2),
            "launches": cnt, "rotating_sets": sets}


def cpu_baseline(cfg_name, seed=0):
    """The NumPy oracle's learn() on the same workload, one full step, host cores."""
    sys.path.insert(0, ROOT)
    from oracle import ppo_np as P
    _, T, N, D, A, cont, pt, ptr = CONFIGS[cfg_name]
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
    adam = P.new_adam_state(params, names)
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    P.learn(params, adam, (obs, nobs, act, rew, te, tr), P.Hyper(), 3e-4, cont,
            rng=np.random.RandomState(42))
    dt = time.perf_counter() - t0
    return {"value": round(T * N / dt, 1), "unit": "env-steps/s", "cores": int(threads),
            "kind": "port",
            "sample": f"one full learn() of the same workload (T={T}, N={N}: old-policy eval, "
                      f"GAE, 4x8 minibatch steps) by the NumPy float32 oracle "
                      f"(oracle/ppo_np.py), {dt:.2f} s",
            "seconds": round(dt, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cartpole4096", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gae-roofline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no per-kernel HIP events in the timed region (no roofline)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    import diamond
    model, T, N, D, A, cont, pt, ptr = CONFIGS[args.config]
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=N, verbose=False, total_steps=10 ** 12)
    agent = Agent(None, cfg, envs=SpecEnvs(D, A, cont))
    assert agent._learner.fused, "benchmark must exercise the fused HIP path"
    ro, _ = synth_rollout(T, N, D, A, cont, pt, ptr, seed=rank, device=device)
    torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        agent.learn_device(ro)
    torch.cuda.synchronize(device)
    h = agent._learner.handle
    hs = agent._learner.host_seconds

    def timed_pass(instrument: bool):
        """K learns between barrier + synchronize brackets; max wall time over ranks."""
        h.set_timing(instrument)
        for k in ("perms", "enqueue", "draft_start"):
            hs[k] = 0.0
        hs["calls"] = 0
        hs["lookahead_hits"] = 0
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            agent.learn_device(ro)
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # Pass A (the reported throughput): no per-launch events in the stream.
    elapsed = timed_pass(False)
    host = {k: round(hs[k] / max(hs["calls"], 1) * 1e3, 4) for k in ("perms", "enqueue",
                                                                      "draft_start")}
    hits = hs["lookahead_hits"]
    # Pass B (the per-kernel table and the roofline): the same K learns with a HIP event pair
    # recorded on the launch stream around every kernel; the markers cost stream time, so this
    # pass's wall time is reported separately and never as the throughput.
    from diamond import _native as NN
    timing = {k: (0.0, 0) for k in NN.TIMING_CLASSES}
    elapsed_instr = None
    if not args.no_kernel_timing:
        elapsed_instr = timed_pass(True)
        timing = h.timing()
    h.set_timing(False)
    loss_trace = agent.learn_trace()

    B_global = T * N * world
    value = B_global * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3
    # dominant kernel by device time in the timed region
    dom = max(timing, key=lambda k: timing[k][0])
    f_eval_full, f_eval_v, f_mb = flops_per_sample(D, A)
    mb = T * N // cfg.num_minibatches
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
                tr = json.load(open(pmc)).get(args.config, {}).get(dom)
                if tr is not None:
                    roofline["traffic"] = tr
            except Exception:
                pass
    kernel_ms = {k: {"ms_total": round(v[0], 3), "launches": v[1],
                     "us_avg": round(v[0] / v[1] * 1e3, 2) if v[1] else 0.0}
                 for k, v in timing.items() if v[1]}
    dev_ms = sum(v[0] for v in timing.values())

    out = None
    if rank == 0:
        out = {
            "metric": "env-steps/sec (GAE+update) on synthetic [128 x num_envs] buffers",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{model}: learn() = old-policy eval + GAE + adv-norm + "
                                   f"{cfg.num_epochs}x{cfg.num_minibatches} minibatch "
                                   f"Adam steps", "name": args.config,
                       "rollout_steps": T, "num_envs_per_gpu": N, "num_envs_total": N * world,
                       "obs_dim": D, "act_dim": A, "continuous": cont, "hidden": H,
                       "batch_per_learn": B_global, "minibatch": mb * world,
                       "parallelism": f"env-axis dp{world}"},
            "roofline": roofline,
            "kernels": kernel_ms,
            "device_ms_per_step": round(dev_ms / args.steps, 4),
            "instrumented_ms_per_step": (round(elapsed_instr / args.steps * 1e3, 4)
                                         if elapsed_instr else None),
            "host_ms_per_step": host,
            "perm_lookahead_hits": hits,
            "final_loss": float(loss_trace[-1, 0]),
            "device": {"name": torch.cuda.get_device_name(device),
                       "arch": getattr(torch.cuda.get_device_properties(device), "gcnArchName", ""),
                       "compute_units": torch.cuda.get_device_properties(device).multi_processor_count},
        }
    if rank == 0 and world == 1 and not args.no_gae_roofline:
        out["roofline_gae"] = gae_roofline(device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args.config)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
