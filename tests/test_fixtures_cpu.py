"""CPU checks of the reference-produced fixtures and oracle restatements beyond learn():

* the checkpoint written by the REFERENCE's Checkpointer.save (tests/golden/make_golden.py
  make_checkpoint_fixture; reference utils.py:584-600) loads with torch.load(weights_only=True)
  into this build's default network and torch Adam (the GPU continuation is in
  test_gpu_rollout_ckpt.py);
* the tanh-squash extension against its oracle restatement
  (oracle.ppo_np.squashed_normal_logp / squash_action).
"""
import os

import numpy as np
import torch

from conftest import GOLDEN, load_golden

import diamond
from diamond.continuous_ppo import squash_to_space, squashed_log_prob
from oracle import ppo_np as P

CKPT = os.path.join(GOLDEN, "ckpt_cartpole-step000128.pt")


class _Box:
    def __init__(self, shape, low=-np.inf, high=np.inf):
        self.shape, self.low, self.high = tuple(shape), low, high


class _Discrete:
    def __init__(self, n):
        self.n, self.shape = n, ()


def test_reference_checkpoint_loads_weights_only():
    chk = torch.load(CKPT, map_location="cpu", weights_only=True)
    assert set(chk) == {"step", "model_state", "opt_state"} and chk["step"] == 128
    import gym_stub
    from diamond.ppo import ActorCriticNetwork
    net = ActorCriticNetwork(gym_stub.Box(shape=(4,)), gym_stub.Discrete(2),
                             cfg=diamond.PPOConfig())
    sd = net.state_dict()
    assert set(sd) == set(chk["model_state"])          # same keys, incl. the actor_out_layer alias
    opt = torch.optim.Adam(net.parameters(), lr=3e-4, eps=1e-5)
    ck = diamond.utils.Checkpointer()
    ck.load(CKPT, net, opt)
    z = load_golden("ckpt_cartpole_resume.npz")
    steps = {float(st["step"]) for st in opt.state.values()}
    assert steps == {float(z[f"adam/{z['param_names'][0]}/step"]) - 32}  # one learn of 4 x 8 steps


def test_squashed_logp_restatement_and_ratio_invariance():
    rng = np.random.default_rng(0)
    n, A = 4096, 6
    u = rng.normal(0, 2.0, (n, A))
    m0, m1 = rng.normal(0, 1, (n, A)), rng.normal(0, 1, (n, A))
    ls0, ls1 = rng.normal(-0.5, 0.2, (1, A)), rng.normal(-0.5, 0.2, (1, A))
    # the build's torch formula (continuous_ppo.squashed_log_prob) against the restatement
    got = squashed_log_prob(torch.from_numpy(m0), torch.from_numpy(ls0), torch.from_numpy(u)).numpy()
    np.testing.assert_allclose(got, P.squashed_normal_logp(m0, ls0, u), rtol=1e-10, atol=1e-9)
    # the correction is parameter-free: the PPO ratio of the squashed policy equals the Gaussian's
    r_sq = np.exp(P.squashed_normal_logp(m1, ls1, u) - P.squashed_normal_logp(m0, ls0, u))
    lp = lambda m, ls: P.normal_logp_entropy(m, ls, u, dt=np.float64)[0]
    r_g = np.exp(lp(m1, ls1) - lp(m0, ls0))
    np.testing.assert_allclose(r_sq, r_g, rtol=1e-9)
    # env actions: inside the bounds, equal to the restatement
    space = _Box((A,), low=-2.0, high=3.0)
    a = squash_to_space(u.astype(np.float32), space)
    np.testing.assert_allclose(a, P.squash_action(u, -2.0, 3.0), rtol=1e-6, atol=1e-6)
    assert a.min() >= -2.0 and a.max() <= 3.0
