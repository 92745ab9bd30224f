#!/usr/bin/env python3
"""How fast is the CPU baseline (oracle/ppo_torch.py, the restatement bench.py times on the GPU
box) against the reference's own learn() on the same cores?  Runs only where /root/reference
exists (this container): imports the reference under the gymnasium stub the golden fixtures use
(tests/golden/make_golden.py), feeds both the same synthetic C3 experience (T = 128, N = 8192,
LunarLander shapes, BASELINE configs[2]) and times one learn() each, alternating, best of
`--reps`.  The reference is timed, never shipped: nothing on the GPU box runs this.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_baseline_vs_reference.py [--reps 3] [--n 8192]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=8192)
    a = ap.parse_args()
    if not os.path.isdir(REF):
        raise SystemExit("no /root/reference here")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gym_stub
    gym_stub.install()
    sys.path.insert(0, REF)
    import diamond
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))  # bench helpers
    import bench
    from oracle import ppo_np as P
    from oracle import ppo_torch as PT

    T, N, D, A = 128, a.n, 8, 4
    bench.CONFIGS["cmp"] = ("LunarLander-shaped", T, N, D, A, False, 0.02, 0.005, "weak")
    exp, params, names, cont, B = bench._baseline_inputs("cmp")
    obs, nobs, act, rew, te, tr = exp
    # the reference's experience: a list over t of [obs, next_obs, actions, rewards, term, trunc]
    # (ppo.py:165-172, staged by learn() itself at :226-232)
    ref_exp = [[obs[t], nobs[t], act[t].astype(np.int64), rew[t].astype(np.float64), te[t], tr[t]]
               for t in range(T)]
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=N)
    agent = diamond.PPO(lambda: gym_stub.SyntheticEnv(D, A), cfg=cfg)
    threads = torch.get_num_threads()
    t_ref, t_port = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        agent.learn(ref_exp)
        t_ref.append(time.perf_counter() - t0)
        p1 = {k: v.copy() for k, v in params.items()}
        t0 = time.perf_counter()
        PT.learn(p1, exp, P.Hyper(), 3e-4, cont, rng=np.random.RandomState(42))
        t_port.append(time.perf_counter() - t0)
    res = {"cpu": PT.cpu_model(), "torch_threads": threads, "T": T, "N": N,
           "reference_learn_s": [round(x, 3) for x in t_ref],
           "restatement_learn_s": [round(x, 3) for x in t_port],
           "reference_env_steps_per_s_best": round(B / min(t_ref), 1),
           "restatement_env_steps_per_s_best": round(B / min(t_port), 1),
           "restatement_over_reference_time": round(min(t_port) / min(t_ref), 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
