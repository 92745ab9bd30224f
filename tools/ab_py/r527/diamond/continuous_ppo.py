"""ContinuousPPO (Gaussian policy) -- drop-in for reference ``diamond/continuous_ppo.py``.

Same config (continuous_ppo.py:15-37), ``JointNormal`` (:40-47), network with a
state-independent ``actor_log_std`` parameter (:50-111; registered first, so it is the first
entry of ``parameters()``), init without the small-output-layer scaling (:114-121).  The fused
kernels evaluate the unsquashed JointNormal exactly as the reference does (there is no tanh squash
anywhere in the reference: continuous_ppo.py:83-111,276-277).

``ContinuousPPOConfig.tanh_squash`` (default False, an extension beyond the reference; SURVEY §8
f2) makes ``rollout()`` send ``a = tanh(u)`` -- rescaled to the action space's bounds when they
are finite -- to the environment while the experience keeps the Gaussian sample ``u``.  With the
default network the squash is computed on the device by the same act-kernel launch that draws
``u`` (``dppo_act_squash_f32``); a custom ``network_cls`` squashes on the host.  The
squashed policy's log-density is ``log N(u) - sum log(1 - tanh(u)^2)`` (:func:`squashed_log_prob`);
the correction does not depend on the parameters, so it cancels in the PPO ratio and the update
is exactly the unsquashed Gaussian update on ``u`` -- the same fused kernels, no second path.  The
entropy bonus stays the Gaussian one (the squashed entropy has no closed form).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable

import numpy as np
import torch
import torch.nn as nn

from ._spaces import is_box
from .ppo import _AgentBase


@dataclass
class ContinuousPPOConfig:
    total_steps: int = 1_000_000
    rollout_steps: int = 64
    num_envs: int = 16
    lr: float = 3e-4
    adam_eps: float = 1e-5
    decay_lr: bool = False
    gamma: float = 0.99
    gae_lambda: float = 0.95
    num_epochs: int = 4
    num_minibatches: int = 8
    ppo_clip: float = 0.2
    value_loss_weight: float = 1.0
    entropy_beta: float = 0.01
    advantage_norm: bool = True
    grad_norm_clip: float = 0.5
    network_hidden_dim: int = 64
    cuda: bool = False
    seed: int | None = 42
    checkpoint: bool = False
    save_interval: float = 600
    verbose: bool = True
    device_index: int = 0
    # data parallelism over ranks (additive): False = each rank permutes its own envs' samples and
    # global minibatch j is the union of the ranks' local minibatches j; True = every rank draws
    # the reference's permutations of the GLOBAL batch (ppo.py:252-255) and processes its members
    # of each global minibatch, so N ranks reproduce the single-GPU learn() of the global batch
    global_minibatches: bool = False
    # GAE kernel (additive): True = the reference's serial recurrence, bit-exact; False = the
    # chunked affine scan (chunk maps composed in parallel), within 1e-6 of the advantages' scale
    gae_bitexact: bool = True
    tanh_squash: bool = False  # extension: env actions tanh(u), experience keeps u (module doc)


class JointNormal(torch.distributions.Normal):
    def log_prob(self, value: torch.Tensor) -> torch.Tensor:
        """Joint log-probability over all action dimensions (continuous_ppo.py:41-43)."""
        return super().log_prob(value).sum(-1)

    def entropy(self) -> torch.Tensor:
        """Joint entropy over all action dimensions (continuous_ppo.py:45-47)."""
        return super().entropy().sum(-1)


class ContinuousActorCriticNetwork(nn.Module):
    def __init__(self, observation_space, action_space, cfg: ContinuousPPOConfig) -> None:
        super().__init__()
        assert is_box(observation_space), "Only Box obs spaces are supported."
        assert is_box(action_space), "Only Box action spaces are supported."
        hidden_dim = cfg.network_hidden_dim
        act_dim = int(np.prod(action_space.shape))
        self.base = nn.Sequential(
            nn.Linear(int(np.prod(observation_space.shape)), hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh())
        self.actor_mean_head = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, act_dim))
        self.actor_log_std = nn.Parameter(torch.zeros(1, act_dim))
        self.critic_head = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, 1))

    def get_actions(self, observations: np.ndarray, device: torch.device) -> np.ndarray:
        x = torch.as_tensor(observations, dtype=torch.float32, device=device)
        with torch.inference_mode():
            mean = self.actor_mean_head(self.base(x))
            log_std = torch.broadcast_to(self.actor_log_std, mean.shape)
            return JointNormal(loc=mean, scale=log_std.exp()).sample().cpu().numpy()

    def get_values(self, observations: torch.Tensor) -> torch.Tensor:
        with torch.inference_mode():
            values = self.critic_head(self.base(observations))
        return values.squeeze(-1)

    def get_means_log_stds_and_values(self, observations: torch.Tensor):
        x = self.base(observations)
        mean = self.actor_mean_head(x)
        log_std = torch.broadcast_to(self.actor_log_std, mean.shape)
        return mean, log_std, self.critic_head(x).squeeze(-1)


def squashed_log_prob(mean: torch.Tensor, log_std: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """log-density of a = tanh(u), u ~ N(mean, exp(log_std)), summed over action dims:
    log N(u) - sum log(1 - tanh(u)^2), with log(1 - tanh(u)^2) = 2 (log 2 - u - softplus(-2u))
    (stable for large |u|)."""
    base = JointNormal(loc=mean, scale=log_std.exp()).log_prob(u)
    corr = 2.0 * (np.log(2.0) - u - torch.nn.functional.softplus(-2.0 * u))
    return base - corr.sum(-1)


def squash_to_space(u: np.ndarray, action_space) -> np.ndarray:
    """tanh(u), rescaled to [low, high] of a Box with finite bounds (else left in [-1, 1])."""
    a = np.tanh(u)
    low = np.asarray(getattr(action_space, "low", -1.0), dtype=np.float64)
    high = np.asarray(getattr(action_space, "high", 1.0), dtype=np.float64)
    if np.all(np.isfinite(low)) and np.all(np.isfinite(high)):
        a = low + (a + 1.0) * 0.5 * (high - low)
    return a.astype(u.dtype, copy=False)


def network_parameter_init_(network: nn.Module, gain: float = 1.0) -> None:
    """Orthogonal weights and zero biases, no output scaling (continuous_ppo.py:114-121)."""
    with torch.no_grad():
        for m in network.modules():
            if isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=gain)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)


class ContinuousPPO(_AgentBase):
    continuous = True
    default_network = ContinuousActorCriticNetwork
    init_fn = staticmethod(network_parameter_init_)

    def __init__(self, env_fn: Callable[[], Any], cfg: ContinuousPPOConfig = ContinuousPPOConfig(),
                 network_cls: Any = ContinuousActorCriticNetwork, envs=None) -> None:
        self._setup(env_fn, cfg, network_cls, envs)

    def _env_actions(self, actions: np.ndarray) -> np.ndarray:
        if getattr(self.cfg, "tanh_squash", False):
            return squash_to_space(actions, self.envs.single_action_space)
        return actions

    def _squash_spec(self):
        """tanh_squash with the fused sampler: the squash runs in the act kernel
        (dppo_act_squash_f32) -- (low, high) for a Box with finite bounds, else plain tanh."""
        if not getattr(self.cfg, "tanh_squash", False):
            return None
        sp = self.envs.single_action_space
        low = np.asarray(getattr(sp, "low", -1.0), dtype=np.float64)
        high = np.asarray(getattr(sp, "high", 1.0), dtype=np.float64)
        if np.all(np.isfinite(low)) and np.all(np.isfinite(high)):
            return (low, high)
        return True
