"""ContinuousPPO (Gaussian policy) -- drop-in for reference ``diamond/continuous_ppo.py``.

Same config (continuous_ppo.py:15-37), ``JointNormal`` (:40-47), network with a
state-independent ``actor_log_std`` parameter (:50-111; registered first, so it is the first
entry of ``parameters()``), init without the small-output-layer scaling (:114-121).  The fused
kernels evaluate the unsquashed JointNormal exactly as the reference does (there is no tanh squash
anywhere in the reference: continuous_ppo.py:83-111,276-277).
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
