"""NumPy float32 restatement of the reference PPO hot path.  TEST INFRASTRUCTURE ONLY.

Every function cites the reference line(s) it restates.  ``T`` = rollout_steps,
``N`` = num_envs, ``B = T*N``, flat sample index ``i = t*N + n`` (reference ``ppo.py:246-249``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

f32 = np.float32

DISCRETE_NAMES = [
    "base.0.weight", "base.0.bias", "base.2.weight", "base.2.bias",
    "actor_head.0.weight", "actor_head.0.bias", "actor_head.2.weight", "actor_head.2.bias",
    "critic_head.0.weight", "critic_head.0.bias", "critic_head.2.weight", "critic_head.2.bias",
]
CONTINUOUS_NAMES = [
    "actor_log_std",
    "base.0.weight", "base.0.bias", "base.2.weight", "base.2.bias",
    "actor_mean_head.0.weight", "actor_mean_head.0.bias",
    "actor_mean_head.2.weight", "actor_mean_head.2.bias",
    "critic_head.0.weight", "critic_head.0.bias", "critic_head.2.weight", "critic_head.2.bias",
]


@dataclass
class Hyper:
    """The config fields the hot path reads (reference ``ppo.py:15-37``)."""
    gamma: float = 0.99
    gae_lambda: float = 0.95
    num_epochs: int = 4
    num_minibatches: int = 8
    ppo_clip: float = 0.2
    value_loss_weight: float = 1.0
    entropy_beta: float = 0.01
    advantage_norm: bool = True
    grad_norm_clip: float = 0.5
    lr: float = 3e-4
    adam_eps: float = 1e-5


# ---------------------------------------------------------------------------------------------
# GAE  (reference ppo.py:188-222; identical in continuous_ppo.py:200-234, recurrent_ppo.py:265-299)
# ---------------------------------------------------------------------------------------------
def gae(rewards, terms, truncs, values, next_values, gamma=0.99, gae_lambda=0.95):
    """Backward GAE recurrence, op-for-op in float32 (no fused multiply-add):

    nt = 1 - term[t]; ntr = 1 - trunc[t]                                    (ppo.py:202-203)
    delta = (r[t] + f32(gamma) * nv[t] * nt) - v[t]                         (ppo.py:206-210)
    a = delta + f32(gamma*lambda) * nt * ntr * a        (gamma*lambda in double; ppo.py:213-220)
    Advantage starts at 0.0 at t = T-1 (ppo.py:198).
    """
    r = np.asarray(rewards, f32)
    te = np.asarray(terms, f32)
    tr = np.asarray(truncs, f32)
    v = np.asarray(values, f32)
    nv = np.asarray(next_values, f32)
    T = r.shape[0]
    g = f32(gamma)
    c = f32(gamma * gae_lambda)  # Python evaluates gamma*gae_lambda first, in double
    adv = np.zeros_like(r)
    a = np.zeros(r.shape[1:], f32)
    for t in range(T - 1, -1, -1):
        nt = f32(1.0) - te[t]
        ntr = f32(1.0) - tr[t]
        delta = (r[t] + (g * nv[t]) * nt) - v[t]
        a = delta + ((c * nt) * ntr) * a
        adv[t] = a
    return adv


def adv_stats(adv):
    """mean and unbiased std over all T*N advantages (ppo.py:243; torch.std correction=1)."""
    x = np.asarray(adv, np.float64).ravel()
    n = x.size
    mean = x.mean()
    var = ((x - mean) ** 2).sum() / (n - 1) if n > 1 else float("nan")
    return f32(mean), f32(math.sqrt(var))


def normalize_adv(adv):
    """(adv - mean) / (std + 1e-6), float32 (ppo.py:242-243)."""
    mean, std = adv_stats(adv)
    return (np.asarray(adv, f32) - mean) / (std + f32(1e-6))


# ---------------------------------------------------------------------------------------------
# Default networks (ppo.py:53-71,84-96; continuous_ppo.py:63-81,95-111)
# ---------------------------------------------------------------------------------------------
def _lin(x, W, b, dt=f32):
    return (x @ W.T + b).astype(dt)


def forward(params, x, continuous=False, dt=f32):
    """Full actor-critic forward; returns the activations the backward needs.

    base = tanh(L2(tanh(L1 x)))                       (ppo.py:53-58)
    discrete:  logits = Lout(tanh(La base))           (ppo.py:60-64)
    continuous: mean = Lmean(tanh(Lm base)), log_std = actor_log_std broadcast
                                                      (continuous_ppo.py:70-76,107-111)
    value = Lv(tanh(Lc base)).squeeze(-1)             (ppo.py:67-71,95)
    """
    head = "actor_mean_head" if continuous else "actor_head"
    x = np.asarray(x, dt)
    h1 = np.tanh(_lin(x, params["base.0.weight"], params["base.0.bias"], dt))
    h2 = np.tanh(_lin(h1, params["base.2.weight"], params["base.2.bias"], dt))
    ha = np.tanh(_lin(h2, params[f"{head}.0.weight"], params[f"{head}.0.bias"], dt))
    out = _lin(ha, params[f"{head}.2.weight"], params[f"{head}.2.bias"], dt)
    hc = np.tanh(_lin(h2, params["critic_head.0.weight"], params["critic_head.0.bias"], dt))
    v = _lin(hc, params["critic_head.2.weight"], params["critic_head.2.bias"], dt)[..., 0]
    return dict(x=x, h1=h1, h2=h2, ha=ha, hc=hc, out=out, v=v)


def values_only(params, x):
    """get_values: base + critic only (ppo.py:84-89)."""
    x = np.asarray(x, f32)
    h1 = np.tanh(_lin(x, params["base.0.weight"], params["base.0.bias"]))
    h2 = np.tanh(_lin(h1, params["base.2.weight"], params["base.2.bias"]))
    hc = np.tanh(_lin(h2, params["critic_head.0.weight"], params["critic_head.0.bias"]))
    return _lin(hc, params["critic_head.2.weight"], params["critic_head.2.bias"])[..., 0]


def log_softmax(z, dt=f32):
    """Categorical(logits) normalisation: z - logsumexp(z) (torch distributions/categorical.py:78)."""
    z = np.asarray(z, dt)
    mx = z.max(-1, keepdims=True)
    lse = mx + np.log(np.exp(z - mx).sum(-1, keepdims=True, dtype=dt)).astype(dt)
    return (z - lse).astype(dt)


def categorical_logp_entropy(logits, actions, dt=f32):
    """log_prob (categorical.py:156) and entropy with log p clamped at finfo.min (:158-162)."""
    lp = log_softmax(logits, dt)
    p = np.exp(lp)
    logp = np.take_along_axis(lp, np.asarray(actions, np.int64)[..., None], -1)[..., 0]
    lpc = np.maximum(lp, np.finfo(dt).min)
    ent = -(lpc * p).sum(-1)
    return logp.astype(dt), ent.astype(dt), p, lp


LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))


def normal_logp_entropy(mean, log_std, actions, dt=f32):
    """JointNormal (continuous_ppo.py:40-47) over torch Normal (distributions/normal.py:88-116):
    log_prob = sum_a [-(x-mu)^2/(2 sigma^2) - log sigma - log sqrt(2 pi)],
    entropy  = sum_a [0.5 + 0.5 log(2 pi) + log sigma], sigma = exp(log_std)."""
    sigma = np.exp(np.asarray(log_std, dt))
    var = sigma * sigma
    log_scale = np.log(sigma)
    x = np.asarray(actions, dt)
    lp = (-((x - mean) ** 2) / (2 * var) - log_scale - dt(LOG_SQRT_2PI)).sum(-1)
    ent = np.broadcast_to(dt(0.5 + 0.5 * math.log(2 * math.pi)) + log_scale, mean.shape).sum(-1)
    return lp.astype(dt), ent.astype(dt)


def old_policy(params, obs, actions, next_obs, continuous=False):
    """Old-policy evaluation under inference_mode (ppo.py:235-238; continuous_ppo.py:247-250)."""
    f = forward(params, obs, continuous)
    if continuous:
        logp, _ = normal_logp_entropy(f["out"], params["actor_log_std"], actions)
    else:
        logp, _, _, _ = categorical_logp_entropy(f["out"], actions)
    nv = values_only(params, next_obs)
    return logp, f["v"], nv, f["out"]


# ---------------------------------------------------------------------------------------------
# Loss + analytic backward for one minibatch (ppo.py:261-283; continuous_ppo.py:273-295)
# ---------------------------------------------------------------------------------------------
def minibatch_loss_grads(params, obs, actions, old_logp, adv, ret, hp: Hyper, continuous=False,
                         m_total=None, dt=f32):
    """Returns (loss, components, grads).  ``m_total`` is the size the means divide by
    (the global minibatch size; equals len(obs) on one device).  ``dt=np.float64`` evaluates the
    same formulas in double precision: the exact-math yardstick the parity tests measure both
    float32 implementations against at full minibatch sizes (65,536-131,072-term sums)."""
    m = obs.shape[0] if m_total is None else m_total
    f32 = dt  # noqa: N806 -- every float32 cast below follows the requested precision
    if dt is not np.float32:
        params = {k: np.asarray(v, dt) for k, v in params.items()}
    head = "actor_mean_head" if continuous else "actor_head"
    f = forward(params, obs, continuous, dt)
    eps = f32(hp.ppo_clip)
    if continuous:
        logp, ent = normal_logp_entropy(f["out"], params["actor_log_std"], actions, dt)
    else:
        logp, ent, p, lp = categorical_logp_entropy(f["out"], actions, dt)
    adv = np.asarray(adv, f32)
    ret = np.asarray(ret, f32)
    ratio = np.exp(logp - np.asarray(old_logp, f32))                       # ppo.py:266
    rc = np.clip(ratio, f32(1.0) - eps, f32(1.0) + eps)
    u = -adv * ratio                                                        # ppo.py:267
    w = -adv * rc                                                           # ppo.py:268-269
    l_pi = np.maximum(u, w).sum(dtype=np.float64) / m                      # ppo.py:270
    l_v = 0.5 * ((f["v"] - ret) ** 2).sum(dtype=np.float64) / m           # ppo.py:272
    h = ent.sum(dtype=np.float64) / m                                     # ppo.py:274
    loss = l_pi + hp.value_loss_weight * l_v - hp.entropy_beta * h        # ppo.py:276-280

    # d max(u, w): torch maximum splits the gradient on ties (derivatives.yaml 'maximum');
    # clamp passes the gradient on the closed interval [1-eps, 1+eps].
    inr = ((ratio >= f32(1.0) - eps) & (ratio <= f32(1.0) + eps)).astype(f32)
    gu = np.where(u > w, 1.0, np.where(u == w, 0.5, 0.0)).astype(f32)
    gw = np.where(w > u, 1.0, np.where(u == w, 0.5, 0.0)).astype(f32)
    dratio = (gu * -adv + gw * -adv * inr) / f32(m)
    dlogp = dratio * ratio
    dv = f32(hp.value_loss_weight) * (f["v"] - ret) / f32(m)
    grads = {}
    if continuous:
        mean = f["out"]
        sigma = np.exp(params["actor_log_std"]).astype(f32)
        x = np.asarray(actions, f32)
        z = (x - mean) / sigma
        dout = dlogp[:, None] * (x - mean) / (sigma * sigma)
        grads["actor_log_std"] = ((dlogp[:, None] * (z * z - 1)).sum(0, keepdims=True)
                                  - f32(hp.entropy_beta)).astype(f32)
    else:
        onehot = np.zeros_like(p)
        onehot[np.arange(len(actions)), np.asarray(actions, np.int64)] = 1
        dout = dlogp[:, None] * (onehot - p) + f32(hp.entropy_beta / m) * p * (lp + ent[:, None])
    dout = dout.astype(f32)
    # heads
    grads[f"{head}.2.weight"] = dout.T @ f["ha"]
    grads[f"{head}.2.bias"] = dout.sum(0)
    dza = (dout @ params[f"{head}.2.weight"]) * (1 - f["ha"] ** 2)
    grads["critic_head.2.weight"] = (dv[:, None] * f["hc"]).sum(0, keepdims=True)
    grads["critic_head.2.bias"] = np.array([dv.sum()], f32)
    dzc = (dv[:, None] * params["critic_head.2.weight"][0][None, :]) * (1 - f["hc"] ** 2)
    grads[f"{head}.0.weight"] = dza.T @ f["h2"]
    grads[f"{head}.0.bias"] = dza.sum(0)
    grads["critic_head.0.weight"] = dzc.T @ f["h2"]
    grads["critic_head.0.bias"] = dzc.sum(0)
    dh2 = dza @ params[f"{head}.0.weight"] + dzc @ params["critic_head.0.weight"]
    dz2 = dh2 * (1 - f["h2"] ** 2)
    grads["base.2.weight"] = dz2.T @ f["h1"]
    grads["base.2.bias"] = dz2.sum(0)
    dz1 = (dz2 @ params["base.2.weight"]) * (1 - f["h1"] ** 2)
    grads["base.0.weight"] = dz1.T @ f["x"]
    grads["base.0.bias"] = dz1.sum(0)
    grads = {k: np.asarray(v, f32) for k, v in grads.items()}
    comps = dict(loss_policy=l_pi, loss_value=l_v, entropy=h)
    return float(loss), comps, grads


# ---------------------------------------------------------------------------------------------
# clip_grad_norm_ (ppo.py:284 -> torch nn/utils/clip_grad.py:96,106,165,169) and Adam
# (ppo.py:135,285 -> torch optim/adam.py:_single_tensor_adam, the CPU path)
# ---------------------------------------------------------------------------------------------
def clip_grad_norm(grads, names, max_norm):
    norms = np.array([np.sqrt((grads[n].astype(np.float64) ** 2).sum()) for n in names], f32)
    total = f32(np.sqrt((norms.astype(np.float64) ** 2).sum()))
    coef = f32(max_norm) / (total + f32(1e-6))
    coef = min(coef, f32(1.0))
    for n in names:
        grads[n] = (grads[n] * coef).astype(f32)
    return float(total), float(coef)


def adam_step(params, grads, state, names, lr, eps, beta1=0.9, beta2=0.999):
    """step += 1; m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2; denom = sqrt(v)/sqrt(bc2) + eps;
    p -= (lr/bc1) m/denom   (adam.py:414,457,476,531-547)."""
    state["step"] += 1
    step = float(state["step"])
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    step_size = lr / bc1
    bc2_sqrt = bc2 ** 0.5
    w = f32(1 - beta1)
    for n in names:
        g = grads[n]
        m = state["m"][n]
        # torch lerp: weight < 0.5 -> self + weight * (end - self)
        m = (m + w * (g - m)).astype(f32)
        v = (state["v"][n] * f32(beta2) + f32(1 - beta2) * g * g).astype(f32)
        denom = (np.sqrt(v) / f32(bc2_sqrt) + f32(eps)).astype(f32)
        params[n] = (params[n] + f32(-step_size) * (m / denom)).astype(f32)
        state["m"][n], state["v"][n] = m, v


def linear_lr_factor_step(lr_now, last_epoch, total_iters, start=1.0, end=1.0):
    """One LinearLR.step() (torch optim/lr_scheduler.py LinearLR.get_lr, recursive form);
    ``last_epoch`` is the epoch index AFTER increment.  ppo.py:137-142,287."""
    if last_epoch == 0:
        return lr_now * start
    if last_epoch > total_iters:
        return lr_now
    return lr_now * (1.0 + (end - start) / (total_iters * start + (last_epoch - 1) * (end - start)))


def new_adam_state(params, names):
    return {"step": 0, "m": {n: np.zeros_like(params[n]) for n in names},
            "v": {n: np.zeros_like(params[n]) for n in names}}


# ---------------------------------------------------------------------------------------------
# learn()  (ppo.py:224-287; continuous_ppo.py:236-299)
# ---------------------------------------------------------------------------------------------
def learn(params, adam, experience, hp: Hyper, lr, continuous=False, perms=None, rng=None,
          record=False):
    """One learn() call.  ``experience`` is (obs, next_obs, actions, rewards, terms, truncs)
    stacked [T, N, ...] arrays; ``perms`` an optional [E, B] permutation (otherwise drawn
    from ``rng`` -- a numpy RandomState -- as ``np.random.permutation`` would, ppo.py:254)."""
    names = CONTINUOUS_NAMES if continuous else DISCRETE_NAMES
    obs, next_obs, actions, rewards, terms, truncs = experience
    obs = np.asarray(obs, f32)
    next_obs = np.asarray(next_obs, f32)
    T, N = obs.shape[:2]
    B = T * N
    logp, values, nvals, _ = old_policy(params, obs, actions, next_obs, continuous)
    adv = gae(rewards, terms, truncs, values, nvals, hp.gamma, hp.gae_lambda)     # ppo.py:240
    ret = values + adv                                                               # ppo.py:241
    if hp.advantage_norm:
        adv = normalize_adv(adv)                                                     # ppo.py:243
    fl = lambda x: np.asarray(x).reshape(B, *np.asarray(x).shape[2:])               # ppo.py:246-249
    obs_f, logp_f, act_f, adv_f, ret_f = fl(obs), fl(logp), fl(actions), fl(adv), fl(ret)
    mb = B // hp.num_minibatches
    if perms is None:
        perms = np.stack([rng.permutation(B) for _ in range(hp.num_epochs)])        # ppo.py:254
    idx = np.asarray(perms).reshape(hp.num_epochs, hp.num_minibatches, mb)          # ppo.py:255
    trace = {"loss": [], "norm": [], "grads": [], "params": [], "comps": []}
    for e in range(hp.num_epochs):
        for j in range(hp.num_minibatches):
            ii = idx[e, j]
            loss, comps, grads = minibatch_loss_grads(params, obs_f[ii], act_f[ii], logp_f[ii],
                                                      adv_f[ii], ret_f[ii], hp, continuous)
            if record:
                trace["grads"].append(np.concatenate([grads[n].ravel() for n in names]))
            norm, _ = clip_grad_norm(grads, names, hp.grad_norm_clip)
            adam_step(params, grads, adam, names, lr, hp.adam_eps)
            trace["loss"].append(loss)
            trace["norm"].append(norm)
            trace["comps"].append(comps)
            if record:
                trace["params"].append(np.concatenate([params[n].ravel() for n in names]))
    trace.update(old_logp=logp, values=values, next_values=nvals, adv_raw=None)
    return trace


# ---------------------------------------------------------------------------------------------
# tanh-squashed Gaussian.  The reference has NO squash (continuous_ppo.py:83-111
# sample and score the raw Gaussian); BASELINE names a "tanh-squash kernel path" for HalfCheetah,
# which this build offers as an opt-in extension (ContinuousPPOConfig.tanh_squash).  Restated here
# so the extension has a CPU yardstick: env action and log-density of a = tanh(u).
# ---------------------------------------------------------------------------------------------
def squash_action(u, low, high):
    """Env action for the Gaussian sample u: tanh(u) rescaled from [-1, 1] to [low, high]."""
    u = np.asarray(u, np.float64)
    return low + (np.tanh(u) + 1.0) * 0.5 * (high - low)


def squashed_normal_logp(mean, log_std, u):
    """log-density of a = tanh(u), u ~ N(mean, exp(log_std)), summed over action dims, in float64:
    log N(u; mean, sigma) - sum_a log(1 - tanh(u_a)^2) (change of variables)."""
    mean = np.asarray(mean, np.float64)
    log_std = np.asarray(log_std, np.float64)
    u = np.asarray(u, np.float64)
    sigma = np.exp(log_std)
    base = (-((u - mean) ** 2) / (2 * sigma * sigma) - log_std - LOG_SQRT_2PI).sum(-1)
    return base - np.log1p(-np.tanh(u) ** 2).sum(-1)
