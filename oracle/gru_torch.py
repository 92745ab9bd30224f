"""Float64 PyTorch-CPU restatement of RecurrentPPO's minibatch loss and gradient -- the INTENDED
semantics of reference diamond/recurrent_ppo.py.  TEST INFRASTRUCTURE ONLY.

The reference cannot run (GRUCore.forward evaluates ``hx or torch.zeros(...)`` and
``dones or ...`` on multi-element tensors, recurrent_ppo.py:78-79, raising RuntimeError for every
num_envs: SURVEY.md §3.5, §8(c)), so no golden trace exists.  This restates what its code says it
does, evaluated in float64 with autograd as the yardstick of the fused HIP kernel (gru.hip):

* ``RecurrentActorCriticNetwork`` (:94-149): base Linear(D, 64) + tanh; ``GRUCore`` (:41-91) = a
  torch GRU cell stepped over t with the hidden state zeroed where ``dones[t]`` (:82-87);
  actor / critic heads Linear(16, 64) tanh Linear(64, A | 1) on the GRU output.
* ``learn`` (:301-367): the full [T, N] sequence recomputed from the rollout's initial hidden
  state (:313, :337), flattened t-major (:340-341), the minibatch's samples selected, the PPO loss
  (:343-356, as ppo.py:264-280), backward.

Parameters: dict name -> numpy array in ``named_parameters()`` order (GRU_NAMES).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

GRU_NAMES = ["base.0.weight", "base.0.bias", "gru.weight_ih_l0", "gru.weight_hh_l0",
             "gru.bias_ih_l0", "gru.bias_hh_l0", "actor_head.0.weight", "actor_head.0.bias",
             "actor_head.2.weight", "actor_head.2.bias", "critic_head.0.weight",
             "critic_head.0.bias", "critic_head.2.weight", "critic_head.2.bias"]


def sequence(p, obs, prev_dones, hx0):
    """Heads over the whole rollout: logits [T, N, A], values [T, N] (recurrent_ppo.py:127-149)."""
    T = obs.shape[0]
    G = p["gru.weight_hh_l0"].shape[1]
    x1 = torch.tanh(F.linear(obs, p["base.0.weight"], p["base.0.bias"]))
    gi = F.linear(x1, p["gru.weight_ih_l0"], p["gru.bias_ih_l0"])
    h = hx0
    outs = []
    for t in range(T):
        h = h * (~prev_dones[t]).to(h.dtype)[:, None]          # hx[:, dones[t]] = 0 (:84)
        gh = F.linear(h, p["gru.weight_hh_l0"], p["gru.bias_hh_l0"])
        r = torch.sigmoid(gi[t, :, :G] + gh[:, :G])
        z = torch.sigmoid(gi[t, :, G:2 * G] + gh[:, G:2 * G])
        n = torch.tanh(gi[t, :, 2 * G:] + r * gh[:, 2 * G:])
        h = (1 - z) * n + z * h
        outs.append(h)
    ho = torch.stack(outs)
    ya = torch.tanh(F.linear(ho, p["actor_head.0.weight"], p["actor_head.0.bias"]))
    logits = F.linear(ya, p["actor_head.2.weight"], p["actor_head.2.bias"])
    yc = torch.tanh(F.linear(ho, p["critic_head.0.weight"], p["critic_head.0.bias"]))
    values = F.linear(yc, p["critic_head.2.weight"], p["critic_head.2.bias"]).squeeze(-1)
    return logits, values


def minibatch_grads(params, obs, actions, old_log_probs, advantages, returns, prev_dones, hx0,
                    mb_idx, m_total, clip=0.15, vf=1.0, ent=0.01):
    """(loss sums {policy, value, entropy}, grads dict) in float64 for the samples mb_idx (flat
    t * N + n) of one rollout, divided by m_total (recurrent_ppo.py:337-358)."""
    p = {k: torch.tensor(np.asarray(v, np.float64), requires_grad=True) for k, v in params.items()}
    d = lambda x: torch.as_tensor(np.asarray(x), dtype=torch.float64)
    logits, values = sequence(p, d(obs), torch.as_tensor(np.asarray(prev_dones, bool)), d(hx0))
    A = logits.shape[-1]
    lg = logits.reshape(-1, A)[mb_idx]
    v = values.reshape(-1)[mb_idx]
    act = torch.as_tensor(np.asarray(actions).reshape(-1)[mb_idx], dtype=torch.int64)
    dist = torch.distributions.Categorical(logits=lg)
    ratio = torch.exp(dist.log_prob(act) - d(old_log_probs).reshape(-1)[mb_idx])
    adv = d(advantages).reshape(-1)[mb_idx]
    ret = d(returns).reshape(-1)[mb_idx]
    pi = torch.maximum(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip, 1 + clip)).sum()
    vl = (0.5 * (v - ret) ** 2).sum()
    en = dist.entropy().sum()
    loss = (pi + vf * vl - ent * en) / m_total
    loss.backward()
    sums = np.array([pi.item(), vl.item(), en.item()])
    return sums, {k: t.grad.numpy().copy() for k, t in p.items()}
