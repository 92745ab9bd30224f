"""GPU checks of the rollout-side and checkpoint rows against the reference.

* f1 -- the fused actor (csrc/mlp.hip act_kernel, replaces get_actions ppo.py:73-82 /
  continuous_ppo.py:83-93): its pre-sampling head outputs (dppo_actor_forward_f32) against the
  logits / Gaussian means the REFERENCE computed for the same observations and weights (captured
  in the golden traces) and against the oracle's forward; and its draws reproduced exactly from
  the documented Philox4x32-10 stream (inverse CDF / Box-Muller, restated below in NumPy) on the
  oracle's probabilities.
* f3 -- resuming from a checkpoint written by the REFERENCE's Checkpointer.save (fixture from
  tests/golden/make_golden.py): load it weights-only into a fresh agent, learn() the next rollout,
  and compare with the reference agent that did the same.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import diamond
from diamond import _native as N
from oracle import ppo_np as P

from conftest import GOLDEN, load_golden
from gpu_helpers import dev, stream
from test_gpu_parity import experience, flat_params, make_agent

M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c, key):
    """NumPy restatement of the kernel's Philox4x32-10 (csrc/mlp.hip philox4x32)."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint64) & M32 for x in c)
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & M32,
                          (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & M32)
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return c0, c1, c2, c3


def u01(x):
    return (((np.asarray(x, np.uint64) >> np.uint64(8)).astype(np.float64) + 0.5)
            / 16777216.0)


def actor_heads(agent, obs):
    L = agent._learner
    o = torch.from_numpy(np.ascontiguousarray(obs, np.float32)).to(dev())
    n = o.shape[0]
    out = torch.empty((n, L.A), device=dev())
    N.check(L.handle.lib.dppo_actor_forward_f32(L.handle.h, L.flat.flat.data_ptr(), o.data_ptr(),
                                                n, out.data_ptr(), stream()))
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("name", ["cartpole_small", "lunar_medium", "cheetah_small",
                                  "pendulum_medium"])
def test_actor_heads_match_reference_forward(name):
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, _ = (int(x) for x in z["dims"])
    agent = make_agent(z)
    obs = z["exp0/obs"].reshape(T * Nn, D)
    got = actor_heads(agent, obs)
    ref = z["old/means" if cont else "old/logits"][0].reshape(T * Nn, A)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-5)
    params = {n: z["init/" + n] for n in z["param_names"]}
    np.testing.assert_allclose(got, P.forward(params, obs, bool(cont))["out"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("cont", [False, True])
def test_fused_draws_are_the_documented_philox_stream(cont):
    """dppo_act_f32's actions, reproduced from Philox4x32-10 (key = seed, counter = (sample index,
    call counter)) on the ORACLE's distribution: discrete = inverse CDF of softmax(logits) at
    u01(c0); continuous = mean + exp(log_std) * Box-Muller(u01(c0), u01(c1)) (pairs (c0,c1),
    (c2,c3) per block of 4 action dims, block k0 xor-ed into the counter's high word)."""
    name = "cheetah_small" if cont else "lunar_medium"
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, c_, _ = (int(x) for x in z["dims"])
    agent = make_agent(z)
    L = agent._learner
    obs = np.ascontiguousarray(z["exp0/obs"].reshape(T * Nn, D), np.float32)
    n = obs.shape[0]
    o = torch.from_numpy(obs).to(dev())
    act = torch.empty((n, A) if cont else (n,), dtype=torch.float32 if cont else torch.int32,
                      device=dev())
    seed, counter = 0x1234_5678_9ABC_DEF1, 77
    N.check(L.handle.lib.dppo_act_f32(L.handle.h, L.flat.flat.data_ptr(), o.data_ptr(), n, seed,
                                      counter, act.data_ptr(), stream()))
    torch.cuda.synchronize()
    got = act.cpu().numpy()
    params = {k: z["init/" + k] for k in z["param_names"]}
    out = P.forward(params, obs, cont)["out"].astype(np.float64)
    key = (seed & 0xFFFFFFFF, seed >> 32)
    i = np.arange(n, dtype=np.uint64)
    if not cont:
        c = philox4x32_10((i & M32, i >> np.uint64(32), np.full(n, counter), np.zeros(n)), key)
        u = u01(c[0])
        p = np.exp(out - out.max(1, keepdims=True))
        cdf = np.cumsum(p / p.sum(1, keepdims=True), axis=1)
        want = np.minimum((u[:, None] >= cdf).sum(1), A - 1)
        margin = np.abs(u[:, None] - cdf[:, :-1]).min(1)
        clear = margin > 1e-5          # away from a CDF boundary by more than fp32 noise
        assert clear.mean() > 0.99
        assert np.array_equal(got[clear], want[clear])
    else:
        want = oracle_gaussian_draws(out, params["actor_log_std"], seed, counter)
        np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)


def oracle_gaussian_draws(out, log_std, seed, counter):
    """The continuous sampler's draws restated: mean + exp(log_std) * Box-Muller on the Philox
    stream (pairs (c0,c1), (c2,c3) per block of 4 action dims, block k0 xor-ed into the counter's
    high word), from the oracle's means ``out`` [n][A]."""
    n, A = out.shape
    key = (seed & 0xFFFFFFFF, seed >> 32)
    i = np.arange(n, dtype=np.uint64)
    ls = np.asarray(log_std, np.float64).reshape(A)
    want = np.empty((n, A))
    for k0 in range(0, A, 4):
        c = philox4x32_10((i & M32, (i >> np.uint64(32)) ^ np.uint64(k0 << 24),
                           np.full(n, counter), np.zeros(n)), key)
        for pp in range(2):
            r = np.sqrt(-2.0 * np.log(u01(c[2 * pp])))
            th = 2 * np.pi * u01(c[2 * pp + 1])
            for kk, val in ((k0 + 2 * pp, r * np.cos(th)), (k0 + 2 * pp + 1, r * np.sin(th))):
                if kk < A:
                    want[:, kk] = out[:, kk] + np.exp(ls[kk]) * val
    return want


@pytest.mark.parametrize("name,bounded", [("cheetah_small", True), ("cheetah_small", False),
                                          ("pendulum_medium", True)])
def test_device_tanh_squash_matches_oracle(name, bounded):
    """f2 on the device: dppo_act_squash_f32 draws the Gaussian samples u (the same stream as
    dppo_act_f32) and, in the same launch, the environment's actions.  Both against the oracle:
    u against the Philox restatement on the oracle's means, the env actions against
    oracle.ppo_np.squash_action on the oracle's samples (tolerance: the samples' 1e-4 through
    tanh' <= 1 and the half-range) and, tightly, on the device's own samples."""
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, _, _ = (int(x) for x in z["dims"])
    agent = make_agent(z)
    L = agent._learner
    obs = np.ascontiguousarray(z["exp0/obs"].reshape(T * Nn, D), np.float32)
    n = obs.shape[0]
    params = {k: z["init/" + k] for k in z["param_names"]}
    with torch.no_grad():   # wider samples, so tanh's saturated tails are exercised
        agent.network.actor_log_std.fill_(0.7)
    params["actor_log_std"] = np.full((1, A), 0.7, np.float32)
    if bounded:
        lo = np.linspace(-2.0, -0.25, A).astype(np.float32)
        hi = np.linspace(0.5, 3.0, A).astype(np.float32)
    o = torch.from_numpy(obs).to(dev())
    u = torch.empty((n, A), device=dev())
    env = torch.empty((n, A), device=dev())
    seed, counter = 0xBEEF_0000_1234_5678, 3
    N.check(L.handle.lib.dppo_act_squash_f32(
        L.handle.h, L.flat.flat.data_ptr(), o.data_ptr(), n, seed, counter,
        lo.ctypes.data if bounded else None, hi.ctypes.data if bounded else None, u.data_ptr(),
        env.data_ptr(), stream()))
    torch.cuda.synchronize()
    u, env = u.cpu().numpy(), env.cpu().numpy()
    u_want = oracle_gaussian_draws(P.forward(params, obs, True)["out"].astype(np.float64),
                                   params["actor_log_std"], seed, counter)
    np.testing.assert_allclose(u, u_want, rtol=1e-4, atol=1e-4)
    if bounded:
        half = 0.5 * (hi.astype(np.float64) - lo)
        env_want = P.squash_action(u_want, lo.astype(np.float64), hi.astype(np.float64))
        env_own = P.squash_action(u, lo.astype(np.float64), hi.astype(np.float64))
        assert np.all(env >= lo) and np.all(env <= hi)
    else:
        half = np.ones(A)
        env_want, env_own = np.tanh(u_want), np.tanh(u.astype(np.float64))
        assert np.all(np.abs(env) <= 1.0)
    np.testing.assert_allclose(env, env_want, rtol=0, atol=float(1e-4 * half.max() + 1e-6))
    np.testing.assert_allclose(env, env_own, rtol=0, atol=float(4e-7 * (1 + np.abs(lo).max() if
                                                                        bounded else 1)))
    assert (np.abs(u) > 3).any()  # saturated tails were drawn
    # and the same u as the unsquashed sampler for this (seed, counter)
    u2 = torch.empty((n, A), device=dev())
    N.check(L.handle.lib.dppo_act_f32(L.handle.h, L.flat.flat.data_ptr(), o.data_ptr(), n, seed,
                                      counter, u2.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert np.array_equal(u, u2.cpu().numpy())


def test_resume_from_reference_checkpoint():
    """Checkpointer file written by the reference after one learn(): a fresh agent loads it
    (torch.load(weights_only=True)) and its next learn() matches the reference's resumed learn()."""
    z = load_golden("ckpt_cartpole_resume.npz")
    T, Nn, D, A = 8, 16, 4, 2
    import gym_stub
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nn, verbose=False)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * Nn)
    agent = diamond.PPO(None, cfg, envs=envs)
    agent.load_checkpoint(os.path.join(GOLDEN, "ckpt_cartpole-step000128.pt"))
    np.random.set_state(("MT19937", z["rng_state"].astype(np.uint32), int(z["rng_pos"]), 0, 0.0))
    keys = ("obs", "next_obs", "actions", "rewards", "term", "trunc")
    exp = [[z["exp/" + k][t] for k in keys] for t in range(T)]
    agent.learn(exp)
    tr = agent.learn_trace()
    torch.cuda.synchronize()
    np.testing.assert_allclose(tr[:, 0], z["loss"], rtol=2e-5, atol=2e-5)
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0, atol=5e-6,
                                   err_msg=n)
        st = agent.optimizer.state[p]
        np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), z[f"adam/{n}/exp_avg"],
                                   rtol=1e-3, atol=1e-7, err_msg=n)
        assert float(st["step"]) == float(z[f"adam/{n}/step"])
