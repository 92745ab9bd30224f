"""RecurrentPPO learn() in one rank of a world of `world` processes (gloo process group, every
rank on cuda:0), for tests/test_gpu_recurrent.py.  Each rank learns on its slice of one synthetic
rollout of the global env axis and writes its flat parameters.  Test infrastructure only."""
import os
import sys

import numpy as np


def synth_experience(T, Ng, D, A, G, device, seed=0):
    """One rollout in RecurrentPPO.rollout()'s layout (recurrent_ppo.py:205-263): per step
    [obs (N,D), actions (N,), rewards, terms, truncs, prev_dones (N,), log_probs, values,
    next_values, hx (1,N,G)] for the GLOBAL env axis."""
    import torch
    rng = np.random.default_rng(seed)
    g = lambda x, dt=torch.float32: torch.as_tensor(x, dtype=dt, device=device)
    exp = []
    hx = g(rng.standard_normal((1, Ng, G)) * 0.5)
    for _ in range(T):
        exp.append([g(rng.standard_normal((Ng, D))), g(rng.integers(0, A, Ng), torch.int64),
                    rng.normal(1.0, 1.0, Ng), rng.random(Ng) < 0.05, rng.random(Ng) < 0.02,
                    g(rng.random(Ng) < 0.1, torch.bool), g(-rng.uniform(0.3, 1.0, Ng)),
                    g(rng.standard_normal(Ng)), g(rng.standard_normal(Ng)), hx])
    return exp


def shard(exp, lo, hi):
    out = []
    for row in exp:
        r = [x[lo:hi] for x in row[:9]] + [row[9][:, lo:hi].contiguous()]
        out.append(r)
    return out


def run(rank, world, port, T, Ng, D, A, out_path):
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for p in (os.path.join(root, "diamond-ppo_amd"), os.path.join(root, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["LOCAL_RANK"] = "0"          # every rank on the one GPU
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import diamond
    import gym_stub
    Nl = Ng // world
    cfg = diamond.RecurrentPPOConfig(rollout_steps=T, num_envs=Nl, num_epochs=3,
                                     num_minibatches=1, verbose=False)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * Nl)
    agent = diamond.RecurrentPPO(None, cfg, envs=envs)
    exp = synth_experience(T, Ng, D, A, cfg.gru_hidden_dim, agent.device)
    init = agent.flat.flat.cpu().numpy()
    agent.learn(shard(exp, rank * Nl, (rank + 1) * Nl))
    torch.cuda.synchronize()
    np.savez(out_path, init=init, final=agent.flat.flat.cpu().numpy())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
