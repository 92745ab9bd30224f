#!/usr/bin/env python3
"""Whole-loop rollout + learn() throughput with a synthetic vector env (SURVEY §8 f1 rehearsal).

Gymnasium is absent in this image, so the env is the test stub (tests/golden/gym_stub.py: NumPy
Gaussian observations and rewards, Bernoulli dones) -- the numbers measure the framework's side of
a real training loop (action sampling on the GPU, per-step staging into HBM, learn()), not an
environment.  Compares rollout staging on (RolloutStager: each step copied into the HBM buffer on
a side stream while the envs step) and off (the experience stacked and uploaded inside learn()),
and action sampling by the fused actor kernel (dppo_act_f32) or by the torch module's
get_actions (the reference's path).

    python tools/train_bench.py [--N 4096] [--T 128] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import diamond  # noqa: E402
import gym_stub  # noqa: E402


def run(stage: bool, fused: bool, T: int, N: int, iters: int, D: int = 4, A: int = 2):
    np.random.seed(0)
    torch.manual_seed(0)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * N)
    agent = diamond.PPO(None, diamond.PPOConfig(rollout_steps=T, num_envs=N, verbose=False),
                        envs=envs)
    agent.stage_rollout = stage
    agent.fused_actions = fused
    agent.current_observations, _ = envs.reset(seed=1)
    agent.learn(agent.rollout())  # warm-up
    torch.cuda.synchronize()
    t_roll = t_learn = 0.0
    t0 = time.perf_counter()
    for _ in range(iters):
        a = time.perf_counter()
        exp = agent.rollout()
        b = time.perf_counter()
        agent.learn(exp)
        torch.cuda.synchronize()
        c = time.perf_counter()
        t_roll += b - a
        t_learn += c - b
    el = time.perf_counter() - t0
    return {"stage_rollout": stage, "fused_actions": fused, "env_steps_per_s": round(T * N * iters / el, 1),
            "rollout_ms": round(t_roll / iters * 1e3, 2),
            "learn_incl_staging_ms": round(t_learn / iters * 1e3, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    for stage, fused in ((False, False), (True, False), (False, True), (True, True)):
        print(json.dumps(run(stage, fused, a.T, a.N, a.iters)), flush=True)


if __name__ == "__main__":
    main()
