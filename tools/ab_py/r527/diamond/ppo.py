"""PPO (discrete actions) -- drop-in for reference ``diamond/ppo.py``.

Same ``PPOConfig`` fields and defaults (ppo.py:15-37), same ``ActorCriticNetwork`` module
structure (ppo.py:40-96, so ``torch.manual_seed`` draws the same initial weights and
``state_dict`` keys match), same ``network_cls`` plug-in protocol, same ``rollout`` /
``calculate_advantage`` / ``learn`` / ``train`` surface.  What differs is where ``learn`` runs:
the whole update is one libdppo call on the MI355X (engine.py), and ``calculate_advantage`` is the
gfx950 GAE kernel.  ``cfg.cuda`` is kept for compatibility; the MI355X build always runs on the
GPU and raises if none is present.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from math import sqrt
from typing import Any, Callable

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from ._spaces import is_box, is_discrete, make_vector_env
from .engine import NativeLearner, DeviceRollout, RolloutStager, dist_world, require_gpu, \
    rebind_after_load, stage_experience
from .utils import Checkpointer, Logger, Ticker, Timer


@dataclass
class PPOConfig:
    # the reference's fields, order and defaults (ppo.py:15-37)
    total_steps: int = 1_000_000    # env steps over the whole train() run
    rollout_steps: int = 64         # T: vector-env steps per rollout
    num_envs: int = 16              # N: environments stepped together
    lr: float = 3e-4                # Adam learning rate
    adam_eps: float = 1e-5          # Adam epsilon (added after dividing by sqrt(bias corr.))
    decay_lr: bool = False          # LinearLR from 1.0 to 0.05 over the run
    gamma: float = 0.99             # discount
    gae_lambda: float = 0.95        # GAE lambda
    num_epochs: int = 4             # passes over each rollout
    num_minibatches: int = 8        # optimizer steps per pass
    ppo_clip: float = 0.2           # surrogate ratio clip
    value_loss_weight: float = 1.0  # value-loss coefficient
    entropy_beta: float = 0.01      # entropy-bonus coefficient
    advantage_norm: bool = True     # standardise advantages over the rollout
    grad_norm_clip: float = 0.5     # max global L2 norm of the gradient
    network_hidden_dim: int = 64    # width of the default MLP
    cuda: bool = False              # kept for compatibility (this build always uses the GPU)
    seed: int | None = 42           # seeds numpy's global RNG and torch
    checkpoint: bool = False        # save checkpoints during train()
    save_interval: float = 600      # seconds between saves
    verbose: bool = True            # print the Ticker table
    device_index: int = 0           # GPU ordinal (additive; LOCAL_RANK wins under torchrun)
    # data parallelism over ranks (additive): False = each rank permutes its own envs' samples and
    # global minibatch j is the union of the ranks' local minibatches j; True = every rank draws
    # the reference's permutations of the GLOBAL batch (ppo.py:252-255) and processes its members
    # of each global minibatch, so N ranks reproduce the single-GPU learn() of the global batch
    global_minibatches: bool = False
    # GAE kernel (additive): True = the reference's serial recurrence, bit-exact; False = the
    # chunked affine scan (chunk maps composed in parallel), within 1e-6 of the advantages' scale
    gae_bitexact: bool = True


class ActorCriticNetwork(nn.Module):
    """Default actor-critic MLP (reference ppo.py:40-96).  Its parameters live in the flat buffer
    the fused kernels update; the torch methods serve rollout() and custom callers."""

    def __init__(self, observation_space, action_space, cfg: PPOConfig) -> None:
        super().__init__()
        assert is_box(observation_space), "Only Box obs spaces are supported."
        assert is_discrete(action_space), "Only Discrete action spaces are supported."
        hidden_dim = cfg.network_hidden_dim
        self.base = nn.Sequential(
            nn.Linear(int(np.prod(observation_space.shape)), hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh())
        self.actor_head = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, int(action_space.n)))
        self.actor_out_layer = self.actor_head[-1]
        self.critic_head = nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim), nn.Tanh(),
            nn.Linear(hidden_dim, 1))

    def get_actions(self, observations: np.ndarray, device: torch.device) -> np.ndarray:
        """Boltzmann action selection (ppo.py:73-82)."""
        x = torch.as_tensor(observations, dtype=torch.float32, device=device)
        with torch.inference_mode():
            logits = self.actor_head(self.base(x))
        return torch.distributions.Categorical(logits=logits).sample().cpu().numpy()

    def get_values(self, observations: torch.Tensor) -> torch.Tensor:
        with torch.inference_mode():
            values = self.critic_head(self.base(observations))
        return values.squeeze(-1)

    def get_logits_and_values(self, x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        x = self.base(x)
        return self.actor_head(x), self.critic_head(x).squeeze(-1)


def network_parameter_init_(network: nn.Module, gain: float = 1.0) -> None:
    """Orthogonal weights, zero biases, small actor output layer (reference ppo.py:99-108)."""
    with torch.no_grad():
        for m in network.modules():
            if isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=gain)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        if hasattr(network, "actor_out_layer"):
            nn.init.orthogonal_(network.actor_out_layer.weight, gain=0.01)  # type: ignore


class _AgentBase:
    """Shared constructor/learn/train plumbing of PPO and ContinuousPPO."""

    continuous = False
    default_network: type = None
    init_fn = staticmethod(network_parameter_init_)
    stage_rollout = True  # rollout() stages each step into HBM as the envs step (RolloutStager)
    # rollout() samples the default network's actions with the fused actor kernel
    # (dppo_act_f32: same distribution as get_actions, Philox draws instead of torch's); False, or
    # any other network_cls, calls network.get_actions as the reference does
    fused_actions = True

    def _setup(self, env_fn, cfg, network_cls, envs=None):
        self.device = require_gpu(getattr(cfg, "device_index", 0))
        world, rank = dist_world()
        if cfg.seed is not None:                                       # ppo.py:120-122
            # local minibatches: env-axis shards draw decorrelated minibatch orders; global
            # minibatches: every rank draws the same permutations of the global batch
            gmb = getattr(cfg, "global_minibatches", False)
            np.random.seed(cfg.seed + (0 if gmb else rank))
            torch.manual_seed(cfg.seed)
        self.envs = envs if envs is not None else make_vector_env(env_fn, cfg.num_envs)
        obs_space = self.envs.single_observation_space
        act_space = self.envs.single_action_space
        # Built and initialised on the host exactly as the reference's CPU default does (same
        # torch RNG draws), then re-homed into the flat HBM buffer the kernels update.
        self.network = network_cls(obs_space, act_space, cfg=cfg)
        self.init_fn(self.network, gain=sqrt(2.0))                      # ppo.py:133
        obs_dim = int(np.prod(obs_space.shape))
        act_dim = int(np.prod(act_space.shape)) if self.continuous else int(act_space.n)
        self._obs_dim, self._act_dim = obs_dim, act_dim
        self.cfg = cfg
        # Adam over the parameters (ppo.py:135); NativeLearner re-homes them into the flat HBM
        # buffer and binds Adam's exp_avg/exp_avg_sq to the kernels' moment buffers.
        self.optimizer = torch.optim.Adam(self.network.parameters(), lr=cfg.lr, eps=cfg.adam_eps)
        self._learner = NativeLearner(self.network, self.optimizer, cfg, obs_dim, act_dim,
                                      self.continuous, self.device,
                                      network_is_default=type(self.network) is self.default_network)
        self.optimizer._opt_called = True  # the kernels step it; silences LinearLR's order check
        self.lr_scheduler = torch.optim.lr_scheduler.LinearLR(
            self.optimizer, start_factor=1.0, end_factor=0.05 if cfg.decay_lr else 1.0,
            total_iters=cfg.total_steps // (cfg.num_envs * cfg.rollout_steps))
        self.logger = Logger()
        self.timer = Timer()
        self.checkpointer = Checkpointer(folder="models", run_name="default")
        self.ticker = Ticker(cfg.total_steps, cfg.num_envs, cfg.rollout_steps,
                             verbose=cfg.verbose and rank == 0)
        self.current_step = 0
        self._stager = None
        self._staged = None
        base_seed = cfg.seed if cfg.seed is not None else torch.initial_seed()
        self._act_seed = (int(base_seed) * 0x9E3779B97F4A7C15 + rank) & (2 ** 64 - 1)

    def _env_actions(self, actions: np.ndarray) -> np.ndarray:
        """What the environment receives for the sampled actions (identity; ContinuousPPO's
        tanh_squash option overrides it).  The experience always keeps ``actions``."""
        return actions

    def _squash_spec(self):
        """None (the env gets the sampled actions), or the fused sampler's squash argument."""
        return None

    # -- drop-in surface ------------------------------------------------------------------------
    def rollout(self) -> list[list[np.ndarray]]:
        """Collect one rollout across the vector env (reference ppo.py:153-186).  Each step is
        also staged into the SoA HBM buffer on a side stream while the envs step; learn() of the
        returned list then skips the stack-and-upload."""
        experience = []
        observations = self.current_observations
        stager = self._rollout_stager()
        if stager is not None:
            stager.begin()
        squash = self._squash_spec()
        for t in range(self.cfg.rollout_steps):
            if self.fused_actions and self._learner.fused:
                if squash is None:
                    actions = self._learner.act(observations, self._act_seed)
                    env_actions = actions
                else:  # the env action comes out of the same kernel launch
                    actions, env_actions = self._learner.act(observations, self._act_seed,
                                                             squash=squash)
            else:
                actions = self.network.get_actions(observations, device=self.device)
                env_actions = self._env_actions(actions)
            next_observations, rewards, terminations, truncations, infos = self.envs.step(
                env_actions)
            experience.append([observations, next_observations, actions, rewards, terminations,
                               truncations])
            if stager is not None:
                stager.put(t, observations, next_observations, actions, rewards, terminations,
                           truncations)
            dones = np.logical_or(terminations, truncations)
            observations, infos = (self.envs.reset(options={"reset_mask": dones})
                                   if np.any(dones) else (next_observations, infos))
            if self.ticker is not None:
                self.ticker.tick(rewards, dones)
        self.current_observations = observations
        if stager is not None:
            stager.end()
        # what was staged: the list and every array object in it (a list edited afterwards, or
        # arrays replaced in it, is re-staged from its contents by learn(); arrays mutated IN
        # PLACE after rollout() are not detected -- set ``agent.stage_rollout = False`` for that)
        self._staged = ((experience, [id(a) for row in experience for a in row])
                        if stager is not None else None)
        return experience

    def _rollout_stager(self):
        if not self.stage_rollout:
            return None
        if self._stager is None:
            obs_shape = (self._obs_dim,)
            act_shape = (self._act_dim,) if self.continuous else ()
            self._stager = RolloutStager(self.cfg.rollout_steps, self.cfg.num_envs, obs_shape,
                                         act_shape, self.continuous, self.device)
        return self._stager

    def calculate_advantage(self, rewards, terminations, truncations, values, next_values):
        """GAE (reference ppo.py:188-222) on the gfx950 kernel, bit-exact with the reference's
        fp32 op order.  Inputs [T, N] tensors (term/trunc as float 0/1 like the reference, or
        bool/uint8); returns advantages [T, N] float32 on the GPU."""
        dev = self.device
        T, Nn = rewards.shape
        if T != self.cfg.rollout_steps:
            raise ValueError(f"rewards has {T} steps, cfg.rollout_steps is {self.cfg.rollout_steps}")
        f = lambda x: torch.as_tensor(x, device=dev).to(torch.float32).contiguous()
        u8 = lambda x: (torch.as_tensor(x, device=dev) != 0).to(torch.uint8).contiguous()
        r, v, nv = f(rewards), f(values), f(next_values)
        te, tr = u8(terminations), u8(truncations)
        adv = torch.empty_like(r)
        ret = torch.empty_like(r)
        h = self._gae_handle(T, Nn)
        stream = torch.cuda.current_stream(dev).cuda_stream
        N.check(h.lib.dppo_gae_f32(h.h, r.data_ptr(), te.data_ptr(), tr.data_ptr(), v.data_ptr(),
                                   nv.data_ptr(), adv.data_ptr(), ret.data_ptr(),
                                   float(self.cfg.gamma), float(self.cfg.gae_lambda), stream),
                "dppo_gae_f32")
        return adv

    def _gae_handle(self, T, Nn):
        if T == self.cfg.rollout_steps and Nn == self.cfg.num_envs:
            return self._learner.handle
        key = (T, Nn)
        cache = self.__dict__.setdefault("_gae_handles", {})
        if key not in cache:
            d = N.Dims(rollout_steps=T, num_envs=Nn, obs_dim=1, act_dim=1, continuous=0,
                       hidden=64, num_epochs=1, num_minibatches=1, world_size=1, rank=0)
            cache[key] = N.Handle(self.device.index or 0, d)
            if not getattr(self.cfg, "gae_bitexact", True):
                cache[key].set_gae_mode(N.GAE_AFFINE)
        return cache[key]

    def learn(self, experience: list[list[np.ndarray]]) -> None:
        """Update policy and value networks with one rollout (reference ppo.py:224-287)."""
        staged, self._staged = self._staged, None
        if (staged is not None and experience is staged[0]
                and [id(a) for row in experience for a in row] == staged[1]):
            ro = self._stager.finish()
            self.learn_device(ro)
            self._stager.release()
            return
        ro = stage_experience(experience, self.device, self.continuous)
        self.learn_device(ro)

    def learn_device(self, rollout: DeviceRollout, outputs: N.LearnOutputs | None = None) -> None:
        """learn() on a rollout already resident in HBM (the benchmarked hot path)."""
        self._learner.learn(rollout, self.optimizer.param_groups[0]["lr"], outputs)
        self.lr_scheduler.step()                                        # ppo.py:287

    def learn_trace(self) -> np.ndarray:
        """[E*M, 5] {loss, loss_policy, loss_value, entropy, grad_norm} of the last learn()."""
        return self._learner.trace()

    def close(self) -> None:
        """Release the agent's device workspace now (also done when it is garbage-collected):
        waits for the look-ahead permutation drafts still writing its pinned slots first."""
        self._learner.close()
        for h in self.__dict__.get("_gae_handles", {}).values():
            h.close()

    def load_checkpoint(self, path) -> None:
        """Checkpointer.load + re-binding of the Adam state to the kernels' flat buffers."""
        self.checkpointer.load(path, self.network, self.optimizer)
        rebind_after_load(self.optimizer, self._learner.flat, self._learner.m, self._learner.v)

    def train(self) -> None:
        """Train PPO agent (reference ppo.py:289-312)."""
        # Under data parallelism each rank's env shard starts from its own seed (the reference's
        # single process seeds its one vector env with cfg.seed), and only rank 0 writes the
        # (replicated) checkpoints -- ranks never race on one file.
        world, rank = dist_world()
        seed = self.cfg.seed
        if seed is not None and world > 1:
            seed = seed + rank * self.cfg.num_envs
        self.current_observations, _ = self.envs.reset(seed=seed)
        saves = self.cfg.checkpoint and rank == 0
        last_checkpoint_time = time.time()
        total_rollouts = self.cfg.total_steps // (self.cfg.rollout_steps * self.cfg.num_envs)
        env_steps = 0
        for rollout_idx in range(total_rollouts):
            experience = self.rollout()
            self.learn(experience)
            env_steps = (rollout_idx + 1) * self.cfg.rollout_steps * self.cfg.num_envs
            if saves:
                if time.time() - last_checkpoint_time >= self.cfg.save_interval:
                    self.checkpointer.save(env_steps, self.network, self.optimizer)
                    last_checkpoint_time = time.time()
        if saves:
            self.checkpointer.save(env_steps, self.network, self.optimizer)
        self.envs.close()


class PPO(_AgentBase):
    continuous = False
    default_network = ActorCriticNetwork
    init_fn = staticmethod(network_parameter_init_)

    def __init__(self, env_fn: Callable[[], Any], cfg: PPOConfig = PPOConfig(),
                 network_cls: Any = ActorCriticNetwork, envs=None) -> None:
        self._setup(env_fn, cfg, network_cls, envs)
