"""PyTorch-CPU restatement of the reference learn() (diamond/ppo.py:224-287,
continuous_ppo.py:236-299).  TEST / BASELINE INFRASTRUCTURE ONLY.

The reference runs its hot path as PyTorch CPU ops: autograd through the actor-critic MLP,
``torch.distributions``, ``nn.utils.clip_grad_norm_`` and ``torch.optim.Adam`` (the CPU
``_single_tensor_adam``).  ``bench.py`` times this restatement on the GPU box's host cores as the
fair CPU baseline (the reference itself cannot travel to the box); the CPU tests pin it against
the golden traces captured from the reference (tests/test_oracle_golden.py).

Parameters are a dict name -> numpy array in the reference's ``named_parameters()`` order
(oracle.ppo_np.DISCRETE_NAMES / CONTINUOUS_NAMES); the network is evaluated functionally with
``F.linear`` on leaf tensors, which is the same arithmetic as the reference's ``nn.Sequential``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .ppo_np import CONTINUOUS_NAMES, DISCRETE_NAMES, Hyper


def _mlp(p, x, head):
    """base -> (actor head, critic head) (ppo.py:53-71,91-96; continuous_ppo.py:63-81,107-111)."""
    h = torch.tanh(F.linear(x, p["base.0.weight"], p["base.0.bias"]))
    h = torch.tanh(F.linear(h, p["base.2.weight"], p["base.2.bias"]))
    a = torch.tanh(F.linear(h, p[f"{head}.0.weight"], p[f"{head}.0.bias"]))
    out = F.linear(a, p[f"{head}.2.weight"], p[f"{head}.2.bias"])
    c = torch.tanh(F.linear(h, p["critic_head.0.weight"], p["critic_head.0.bias"]))
    v = F.linear(c, p["critic_head.2.weight"], p["critic_head.2.bias"]).squeeze(-1)
    return out, v


def _values(p, x):
    """get_values: base + critic only (ppo.py:84-89)."""
    h = torch.tanh(F.linear(x, p["base.0.weight"], p["base.0.bias"]))
    h = torch.tanh(F.linear(h, p["base.2.weight"], p["base.2.bias"]))
    c = torch.tanh(F.linear(h, p["critic_head.0.weight"], p["critic_head.0.bias"]))
    return F.linear(c, p["critic_head.2.weight"], p["critic_head.2.bias"]).squeeze(-1)


def _dist(p, out, continuous):
    if continuous:
        # JointNormal: independent Normals, log-prob / entropy summed over action dims
        # (continuous_ppo.py:40-47), scale = exp(actor_log_std) broadcast (:109)
        base = torch.distributions.Normal(out, p["actor_log_std"].exp().expand_as(out))
        return (lambda a: base.log_prob(a).sum(-1)), (lambda: base.entropy().sum(-1))
    d = torch.distributions.Categorical(logits=out)
    return d.log_prob, d.entropy


def gae(rewards, terms, truncs, values, next_values, gamma, lam):
    """Backward GAE recurrence over the time axis (ppo.py:188-222)."""
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    a = torch.zeros_like(rewards[0])
    for t in range(T - 1, -1, -1):
        nt = 1.0 - terms[t]
        ntr = 1.0 - truncs[t]
        delta = rewards[t] + gamma * next_values[t] * nt - values[t]
        a = delta + gamma * lam * nt * ntr * a
        adv[t] = a
    return adv


def learn(params: dict, experience, hp: Hyper = Hyper(), lr: float | None = None,
          continuous: bool = False, perms=None, rng=None, adam_state=None):
    """One learn() on the host CPU.  ``experience`` = stacked (obs, next_obs, actions, rewards,
    terms, truncs) [T, N, ...] arrays; ``perms`` [E, B] or drawn from ``rng`` like
    np.random.permutation (ppo.py:254).  Updates ``params`` in place (numpy arrays) and returns
    the per-step {loss, norm} trace."""
    names = CONTINUOUS_NAMES if continuous else DISCRETE_NAMES
    head = "actor_mean_head" if continuous else "actor_head"
    lr = hp.lr if lr is None else lr
    p = {n: torch.from_numpy(np.ascontiguousarray(params[n], np.float32)).requires_grad_(True)
         for n in names}
    opt = torch.optim.Adam([p[n] for n in names], lr=lr, eps=hp.adam_eps)
    if adam_state is not None:
        opt.load_state_dict(adam_state)
    obs, next_obs, actions, rewards, terms, truncs = experience
    obs = torch.as_tensor(np.asarray(obs, np.float32))
    next_obs = torch.as_tensor(np.asarray(next_obs, np.float32))
    acts = torch.as_tensor(np.asarray(actions, np.float32 if continuous else np.int64))
    rew = torch.as_tensor(np.asarray(rewards, np.float32))
    te = torch.as_tensor(np.asarray(terms, np.float32))
    tr = torch.as_tensor(np.asarray(truncs, np.float32))
    T, N = obs.shape[:2]
    B = T * N
    with torch.inference_mode():                                        # ppo.py:235-238
        out, values = _mlp(p, obs, head)
        log_prob, _ = _dist(p, out, continuous)
        old_logp = log_prob(acts)
        next_values = _values(p, next_obs)
        adv = gae(rew, te, tr, values, next_values, hp.gamma, hp.gae_lambda)   # ppo.py:240
        ret = values + adv                                                       # ppo.py:241
        if hp.advantage_norm:
            adv = (adv - adv.mean()) / (adv.std() + 1e-6)                       # ppo.py:243
    flat = lambda x: x.reshape(B, *x.shape[2:]).clone()                  # ppo.py:246-249
    obs_f, acts_f, logp_f, adv_f, ret_f = (flat(obs), flat(acts), flat(old_logp), flat(adv),
                                           flat(ret))
    mb = B // hp.num_minibatches
    if perms is None:
        perms = np.stack([rng.permutation(B) for _ in range(hp.num_epochs)])  # ppo.py:252-254
    idx_all = torch.as_tensor(np.asarray(perms, np.int64)).reshape(hp.num_epochs,
                                                                  hp.num_minibatches, mb)
    trace = {"loss": [], "norm": []}
    params_list = [p[n] for n in names]
    for e in range(hp.num_epochs):
        for j in range(hp.num_minibatches):
            ii = idx_all[e, j]
            out_mb, v_mb = _mlp(p, obs_f[ii], head)                     # ppo.py:261
            log_prob, entropy = _dist(p, out_mb, continuous)
            ratio = torch.exp(log_prob(acts_f[ii]) - logp_f[ii])        # ppo.py:264-266
            a = adv_f[ii]
            l_pi = torch.max(-a * ratio,
                             -a * torch.clamp(ratio, 1.0 - hp.ppo_clip, 1.0 + hp.ppo_clip)).mean()
            l_v = 0.5 * F.mse_loss(v_mb, ret_f[ii])                       # ppo.py:272
            ent = entropy().mean()                                         # ppo.py:274
            loss = l_pi + hp.value_loss_weight * l_v - hp.entropy_beta * ent
            opt.zero_grad()
            loss.backward()
            norm = torch.nn.utils.clip_grad_norm_(params_list, hp.grad_norm_clip)   # ppo.py:284
            opt.step()                                                              # ppo.py:285
            trace["loss"].append(float(loss.detach()))
            trace["norm"].append(float(norm))
    with torch.no_grad():
        for n in names:
            params[n][...] = p[n].numpy()
    trace["adam_state"] = opt.state_dict()
    return trace


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"

