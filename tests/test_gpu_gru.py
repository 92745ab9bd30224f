"""The fused RecurrentPPO minibatch kernel (csrc/gru.hip, dppo_gru_minibatch_grad_f32; SURVEY §8
f4) against the float64 autograd restatement of the reference's intended semantics
(oracle/gru_torch.py: recurrent_ppo.py:41-91, :301-367; the reference itself crashes at :78, so
no golden trace exists).

Tolerances: gradients max|diff| <= 2e-5 x max|g| per tensor group (fp32 sums over up to 1,024
samples and 32 BPTT steps); loss sums rel 1e-5.  learn(): fused vs the torch-autograd path of the
same agent -- parameters within 2e-5 after 2 x 2 Adam steps."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import diamond
from diamond import _native as N
from oracle import gru_torch as GT


def _agent(T, Nn, D, A, **kw):
    import gym_stub
    np.random.seed(0)
    torch.manual_seed(0)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * Nn)
    cfg = diamond.RecurrentPPOConfig(rollout_steps=T, num_envs=Nn, verbose=False, **kw)
    return diamond.RecurrentPPO(None, cfg, envs=envs)


def _data(T, Nn, D, A, G, seed):
    rng = np.random.default_rng(seed)
    return dict(obs=rng.standard_normal((T, Nn, D)).astype(np.float32),
                actions=rng.integers(0, A, (T, Nn)).astype(np.int32),
                old_log_probs=(-rng.uniform(0.2, 1.5, (T, Nn))).astype(np.float32),
                advantages=rng.standard_normal((T, Nn)).astype(np.float32),
                returns=rng.standard_normal((T, Nn)).astype(np.float32),
                prev_dones=(rng.random((T, Nn)) < 0.08),
                hx0=(rng.standard_normal((Nn, G)) * 0.5).astype(np.float32))


@pytest.mark.parametrize("T,Nn,D,A,frac", [(32, 32, 4, 2, 1.0), (16, 20, 7, 3, 0.5),
                                           (8, 3, 17, 6, 0.25), (40, 17, 32, 16, 0.3),
                                           (5, 64, 8, 4, 1.0)])
def test_gru_minibatch_gradient_matches_float64_oracle(T, Nn, D, A, frac):
    agent = _agent(T, Nn, D, A)
    assert agent.gru is not None
    G = agent.cfg.gru_hidden_dim
    with torch.no_grad():   # spread the weights so gates and heads leave their linear range
        for p in agent.network.parameters():
            p.add_(torch.randn_like(p) * 0.3)
    x = _data(T, Nn, D, A, G, seed=T * 100 + Nn)
    B = T * Nn
    m = max(1, int(B * frac))
    mb_idx = np.random.default_rng(7).permutation(B)[:m].astype(np.int32)
    dev = agent.device
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in x.items()}
    t["prev_dones"] = t["prev_dones"].to(torch.uint8)
    batch = N.GruBatch(*[t[k].data_ptr() for k in ("obs", "actions", "old_log_probs",
                                                      "advantages", "returns", "prev_dones",
                                                      "hx0")])
    idx = torch.from_numpy(mb_idx).to(dev)
    hp = N.HParams(gamma=0.99, gae_lambda=0.95, ppo_clip=0.15, value_loss_weight=1.0,
                   entropy_beta=0.01, grad_norm_clip=0.5, adam_beta1=0.9, adam_beta2=0.999,
                   adam_eps=1e-5, advantage_norm=1, lr=3e-4, adam_step=0)
    L = agent.gru.layout
    grad = torch.zeros(L.total + 8, device=dev)
    N.check(agent.gru.lib.dppo_gru_minibatch_grad_f32(
        agent.gru.h, agent.flat.flat.data_ptr(), ctypes.byref(batch), idx.data_ptr(), m, m,
        ctypes.byref(hp), grad.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    g = grad.cpu().numpy()
    params = {n: p.detach().cpu().numpy() for n, p in agent.network.named_parameters()}
    assert list(params) == GT.GRU_NAMES
    sums, ref = GT.minibatch_grads(params, x["obs"], x["actions"], x["old_log_probs"],
                                   x["advantages"], x["returns"], x["prev_dones"], x["hx0"],
                                   mb_idx, m)
    scale = max(np.abs(r).max() for r in ref.values())
    for i, n in enumerate(GT.GRU_NAMES):
        got = g[L.offset[i]:L.offset[i] + L.numel[i]].reshape(ref[n].shape)
        err = np.abs(got - ref[n]).max()
        assert err <= 2e-5 * scale, (n, err, scale)
    np.testing.assert_allclose(g[L.total:L.total + 3], sums, rtol=1e-5, atol=1e-5 * m)
    # deterministic: the same call twice gives the same bits
    g2 = torch.zeros_like(grad)
    N.check(agent.gru.lib.dppo_gru_minibatch_grad_f32(
        agent.gru.h, agent.flat.flat.data_ptr(), ctypes.byref(batch), idx.data_ptr(), m, m,
        ctypes.byref(hp), g2.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(grad, g2)


def test_recurrent_learn_fused_matches_torch_path():
    """Two identical agents learn the same rollout (2 epochs x 2 minibatches): the fused kernel
    path and the torch-autograd path end with the same parameters and Adam state."""
    from dist_scripts.recurrent_dp import synth_experience
    T, Nn, D, A = 16, 24, 6, 3
    res = []
    for fused in (True, False):
        agent = _agent(T, Nn, D, A, num_epochs=2, num_minibatches=2)
        agent.fused_gru = fused
        exp = synth_experience(T, Nn, D, A, agent.cfg.gru_hidden_dim, agent.device, seed=3)
        np.random.seed(5)
        agent.learn(exp)
        torch.cuda.synchronize()
        res.append((agent.flat.flat.cpu().numpy(), agent.m.cpu().numpy()))
    (p1, m1), (p2, m2) = res
    assert np.abs(p1 - p2).max() <= 2e-5
    np.testing.assert_allclose(m1, m2, rtol=1e-3, atol=1e-7)
