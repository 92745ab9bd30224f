"""Shared helpers of the GPU test modules (synthetic rollouts, random default-network parameters,
C-ABI hyper-parameters).  Test infrastructure only."""
import numpy as np
import torch

from diamond import _native as N
from diamond.engine import DeviceRollout

H = 64


def dev():
    return torch.device("cuda", 0)


def stream():
    return torch.cuda.current_stream().cuda_stream


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


class Discrete:
    def __init__(self, n):
        self.n = int(n)


class SpecEnvs:
    """Spaces only: learn() on staged buffers never steps an environment."""

    def __init__(self, D, A, cont):
        self.single_observation_space = Box((D,))
        self.single_action_space = Box((A,)) if cont else Discrete(A)


def synth(T, Nn, D, A, cont, seed):
    rng = np.random.default_rng(seed)
    obs = rng.standard_normal((T, Nn, D), dtype=np.float32)
    nobs = rng.standard_normal((T, Nn, D), dtype=np.float32)
    act = (rng.standard_normal((T, Nn, A), dtype=np.float32) if cont
           else rng.integers(0, A, (T, Nn)).astype(np.int32))
    rew = rng.normal(1.0, 1.0, (T, Nn)).astype(np.float32)
    te = (rng.random((T, Nn)) < (0.0 if cont else 0.02)).astype(np.uint8)
    tr = (rng.random((T, Nn)) < (0.001 if cont else 0.005)).astype(np.uint8)
    g = lambda x: torch.from_numpy(x).to(dev())
    return DeviceRollout(g(obs), g(nobs), g(act), g(rew), g(te), g(tr)), (obs, nobs, act, rew, te, tr)


def random_params(L, names, D, A, cont, rng):
    """Parameters of the default network at a scale that keeps tanh units in their active range
    and the policy away from uniform (so the surrogate's clip and both tie branches occur)."""
    params = {}
    for i, n in enumerate(names):
        shp = (L.rows[i],) if n.endswith("bias") else (L.rows[i], L.cols[i])
        if n == "actor_log_std":
            params[n] = rng.normal(-0.5, 0.2, (1, A)).astype(np.float32)
        elif n.endswith("bias"):
            params[n] = rng.normal(0.0, 0.1, shp).astype(np.float32)
        else:
            params[n] = (rng.standard_normal(shp) * 1.2 / np.sqrt(shp[1])).astype(np.float32)
    flat = np.zeros(L.total, np.float32)
    for i, n in enumerate(names):
        flat[L.offset[i]:L.offset[i] + L.numel[i]] = params[n].ravel()
    return params, flat


def hparams():
    return N.HParams(gamma=0.99, gae_lambda=0.95, ppo_clip=0.2, value_loss_weight=1.0,
                     entropy_beta=0.01, grad_norm_clip=0.5, adam_beta1=0.9, adam_beta2=0.999,
                     adam_eps=1e-5, advantage_norm=1, lr=3e-4, adam_step=0)


def nit_of(m):
    """32-sample steps per workgroup of the two-team kernel (mbstep.hip)."""
    steps = (m + 31) // 32
    G = min(steps, 256)
    return (steps + G - 1) // G


def sample_split(D, A, cont):
    """Whether learn() runs the sample-split kernel (mbwave.hip, mbw_supported) for this shape."""
    if cont and 5 <= A <= 6 and D == 17:
        return True  # the X1 instantiation (HalfCheetah)
    return D <= 32 and (A <= 4 or (A <= 8 and not cont and D <= 16))


def groups_per_wave(m):
    """16-sample groups each wave of the sample-split kernel runs (4 waves per workgroup, one
    workgroup per 64 samples up to 256)."""
    groups = (m + 15) // 16
    G = min((m + 63) // 64, 256)
    return (groups + 4 * G - 1) // (4 * G)


def production_depth(m, D, A, cont):
    return groups_per_wave(m) if sample_split(D, A, cont) else nit_of(m)
