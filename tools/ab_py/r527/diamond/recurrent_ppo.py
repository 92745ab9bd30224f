"""RecurrentPPO (GRU core) -- API-compatible with reference ``diamond/recurrent_ppo.py``.

The reference cannot run: ``GRUCore.forward`` evaluates ``hx or torch.zeros(...)`` and
``dones or ...`` on multi-element tensors (recurrent_ppo.py:78-79), so both ``rollout()`` and
``learn()`` raise ``RuntimeError``.  This module implements the intended
semantics: per-timestep GRU with the hidden state reset where ``dones[t]`` (:82-87), old
log-probs / values / next-values cached during rollout (:219-243), and ``learn`` recomputing the
full [T, N] sequence from the stored initial ``hx`` for every minibatch (:337-341).  The network
runs under torch autograd on the GPU; GAE, advantage normalisation and clip + Adam run in the
gfx950 kernels.  No oracle pins this path beyond the shared GAE (reference broken).

Data parallelism (torchrun, one process per GPU): each rank owns its own envs (seeded
``seed + rank * num_envs``) and permutes its own samples (``np.random`` seeded ``seed + rank``);
global minibatch j is the union of the ranks' local minibatches j.  The advantage statistics are
global (the ranks' {sum, sum^2} all-reduced, ppo.py:243 over the global batch), each rank's loss
is its local mean scaled by 1/world, and the flat gradient is all-reduced (SUM, RCCL under the
"nccl" backend) before the replicated clip + Adam -- so every rank takes the identical step.
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass
from math import sqrt
from typing import Any, Callable

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from ._spaces import is_box, is_discrete, make_vector_env
from .engine import FlatParams, bind_adam_state, adam_step_count, advance_adam_steps, \
    dist_world, require_gpu
from .utils import Checkpointer, Logger, Ticker, Timer


@dataclass
class RecurrentPPOConfig:
    total_steps: int = 1_000_000
    rollout_steps: int = 32
    num_envs: int = 32
    lr: float = 3e-4
    adam_eps: float = 1e-5
    decay_lr: bool = False
    gamma: float = 0.99
    gae_lambda: float = 0.95
    num_epochs: int = 10
    num_minibatches: int = 1
    ppo_clip: float = 0.15
    value_loss_weight: float = 1.0
    entropy_beta: float = 0.01
    advantage_norm: bool = True
    grad_norm_clip: float = 0.5
    network_hidden_dim: int = 64
    gru_hidden_dim: int = 16
    cuda: bool = False
    seed: int | None = 42
    checkpoint: bool = False
    save_interval: float = 600
    verbose: bool = True
    device_index: int = 0
    gae_bitexact: bool = True   # False: the chunked affine-scan GAE kernel (PPOConfig)


class GRUCore(nn.GRU):
    """GRU with per-timestep hidden resets (intended semantics of recurrent_ppo.py:41-91)."""

    def __init__(self, input_dim: int, hidden_dim: int) -> None:
        super().__init__(input_dim, hidden_dim)

    def forward(self, x, hx=None, dones=None):
        seq_length, batch_size = x.shape[:2]
        if hx is None:
            hx = torch.zeros(1, batch_size, self.hidden_size, dtype=x.dtype, device=x.device)
        if dones is None:
            dones = torch.zeros(seq_length, batch_size, dtype=torch.bool, device=x.device)
        outputs = []
        for t in range(seq_length):
            keep = (~dones[t].bool()).to(hx.dtype)[None, :, None]
            hx = hx * keep                                 # hx[:, dones[t]] = 0 (:84)
            out, hx = super().forward(x[t:t + 1], hx)
            outputs.append(out)
        return torch.cat(outputs, dim=0), hx


class RecurrentActorCriticNetwork(nn.Module):
    def __init__(self, observation_space, action_space, cfg: RecurrentPPOConfig) -> None:
        super().__init__()
        assert is_box(observation_space), "Only Box obs spaces are supported."
        assert is_discrete(action_space), "Only Discrete action spaces are supported."
        hd, gd = cfg.network_hidden_dim, cfg.gru_hidden_dim
        self.base = nn.Sequential(nn.Linear(int(np.prod(observation_space.shape)), hd), nn.Tanh())
        self.gru = GRUCore(hd, gd)
        self.actor_head = nn.Sequential(nn.Linear(gd, hd), nn.Tanh(),
                                        nn.Linear(hd, int(action_space.n)))
        self.actor_out_layer = self.actor_head[-1]
        self.critic_head = nn.Sequential(nn.Linear(gd, hd), nn.Tanh(), nn.Linear(hd, 1))

    def get_values(self, observations, hx, dones):
        x = self.base(observations)
        x, hx = self.gru.forward(x, hx, dones)
        return self.critic_head(x).squeeze(-1)

    def get_logits_values_and_hx(self, observations, hx, dones):
        x = self.base(observations)
        x, hx = self.gru.forward(x, hx, dones)
        return self.actor_head(x), self.critic_head(x).squeeze(-1), hx


def network_parameter_init_(network: nn.Module, gain: float = 1.0) -> None:
    with torch.no_grad():
        for m in network.modules():
            if isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=gain)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        if hasattr(network, "actor_out_layer"):
            nn.init.orthogonal_(network.actor_out_layer.weight, gain=0.01)


class RecurrentPPO:
    # learn() runs each minibatch's sequence recompute, loss and BPTT as one fused HIP launch
    # (dppo_gru_minibatch_grad_f32) for the default network at supported shapes; False (or any
    # other network_cls) runs the network under torch autograd on the GPU
    fused_gru = True

    def __init__(self, env_fn: Callable[[], Any], cfg: RecurrentPPOConfig = RecurrentPPOConfig(),
                 network_cls: Any = RecurrentActorCriticNetwork, envs=None) -> None:
        self.device = require_gpu(cfg.device_index)
        world, rank = dist_world()
        if cfg.seed is not None:
            np.random.seed(cfg.seed + rank)
            torch.manual_seed(cfg.seed)   # same initial weights on every rank
        self.envs = envs if envs is not None else make_vector_env(env_fn, cfg.num_envs)
        obs_space, act_space = self.envs.single_observation_space, self.envs.single_action_space
        self.network = network_cls(obs_space, act_space, cfg=cfg)
        network_parameter_init_(self.network, gain=sqrt(2.0))
        self.optimizer = torch.optim.Adam(self.network.parameters(), lr=cfg.lr, eps=cfg.adam_eps)
        self.flat = FlatParams(self.network, self.device)
        self.flat.bind_grads()
        self.m, self.v = bind_adam_state(self.optimizer, self.flat)
        self.optimizer._opt_called = True
        self.lr_scheduler = torch.optim.lr_scheduler.LinearLR(
            self.optimizer, start_factor=1.0, end_factor=0.05 if cfg.decay_lr else 1.0,
            total_iters=cfg.total_steps // (cfg.num_envs * cfg.rollout_steps))
        dims = N.Dims(rollout_steps=cfg.rollout_steps, num_envs=cfg.num_envs, obs_dim=1,
                      act_dim=1, continuous=0, hidden=cfg.network_hidden_dim,
                      num_epochs=cfg.num_epochs, num_minibatches=cfg.num_minibatches,
                      world_size=1, rank=0)
        self.handle = N.Handle(self.device.index or 0, dims)
        self.gru = None
        obs_dim = int(np.prod(obs_space.shape))
        if (type(self.network) is RecurrentActorCriticNetwork and cfg.network_hidden_dim == 64
                and cfg.gru_hidden_dim == 16 and obs_dim <= 32 and int(act_space.n) <= 16):
            gd = N.GruDims(rollout_steps=cfg.rollout_steps, num_envs=cfg.num_envs,
                           obs_dim=obs_dim, act_dim=int(act_space.n), hidden=64, gru_hidden=16)
            self.gru = N.GruHandle(self.device.index or 0, gd)
            L = self.gru.layout
            if L.total != self.flat.total or any(L.offset[i] != o for i, o in
                                                  enumerate(self.flat.offsets)):
                raise RuntimeError("RecurrentActorCriticNetwork layout differs from libdppo's")
        self.last_losses = None
        if not getattr(cfg, "gae_bitexact", True):
            self.handle.set_gae_mode(N.GAE_AFFINE)
        if world > 1:   # replicate rank 0's initial weights (identical seeds: a no-op in practice)
            d = torch.distributed
            if d.get_backend() == "nccl":
                d.broadcast(self.flat.flat, src=0)
            else:
                cpu = self.flat.flat.cpu()
                d.broadcast(cpu, src=0)
                self.flat.flat.copy_(cpu)
        self.logger, self.timer = Logger(), Timer()
        self.checkpointer = Checkpointer(folder="models", run_name="default")
        self.ticker = Ticker(cfg.total_steps, cfg.num_envs, cfg.rollout_steps, verbose=cfg.verbose)
        self.cfg = cfg

    def rollout(self):
        """recurrent_ppo.py:205-263 with tensor-safe hidden-state handling."""
        experience = []
        observations, hx, prev_dones = self.current_observations, self.current_hx, self.prev_dones
        for _ in range(self.cfg.rollout_steps):
            obs_t = torch.as_tensor(observations[None, ...], dtype=torch.float32, device=self.device)
            pd_t = torch.as_tensor(prev_dones[None, ...], dtype=torch.bool, device=self.device)
            with torch.inference_mode():
                logits, values, new_hx = self.network.get_logits_values_and_hx(obs_t, hx, pd_t)
            dist = torch.distributions.Categorical(logits=logits.squeeze(0))
            actions = dist.sample()
            log_probs = dist.log_prob(actions)
            next_observations, rewards, terms, truncs, infos = self.envs.step(actions.cpu().numpy())
            nobs_t = torch.as_tensor(next_observations[None, ...], dtype=torch.float32,
                                     device=self.device)
            with torch.inference_mode():
                next_values = self.network.get_values(nobs_t, new_hx, None)
            experience.append([obs_t.squeeze(0), actions, rewards, terms, truncs, pd_t.squeeze(0),
                               log_probs, values.squeeze(0), next_values.squeeze(0), hx])
            dones = np.logical_or(terms, truncs)
            observations, infos = (self.envs.reset(options={"reset_mask": dones})
                                   if np.any(dones) else (next_observations, infos))
            hx, prev_dones = new_hx, dones
            if self.ticker is not None:
                self.ticker.tick(rewards, dones)
        self.current_observations, self.current_hx, self.prev_dones = observations, hx, prev_dones
        return experience

    def calculate_advantage(self, rewards, terminations, truncations, values, next_values):
        """Shared GAE (recurrent_ppo.py:265-299) on the gfx950 kernel."""
        dev = self.device
        f = lambda x: torch.as_tensor(x, device=dev).to(torch.float32).contiguous()
        u8 = lambda x: (torch.as_tensor(x, device=dev) != 0).to(torch.uint8).contiguous()
        # every operand bound to a name until the launch is enqueued: a temporary's block would go
        # back to the caching allocator at once and could be handed to the next operand's copy
        r, v, nv = f(rewards), f(values), f(next_values)
        te, tr = u8(terminations), u8(truncations)
        adv, ret = torch.empty_like(r), torch.empty_like(r)
        stream = torch.cuda.current_stream(dev).cuda_stream
        N.check(self.handle.lib.dppo_gae_f32(
            self.handle.h, r.data_ptr(), te.data_ptr(), tr.data_ptr(),
            v.data_ptr(), nv.data_ptr(), adv.data_ptr(), ret.data_ptr(), float(self.cfg.gamma),
            float(self.cfg.gae_lambda), stream), "dppo_gae_f32")
        return adv

    def learn(self, experience) -> None:
        """recurrent_ppo.py:301-367 (intended semantics)."""
        cfg, lib, h = self.cfg, self.handle.lib, self.handle.h
        (observations, actions, rewards, terms, truncs, prev_dones, log_probs, values,
         next_values, hx) = zip(*experience)
        observations = torch.stack(observations)
        actions = torch.stack(actions)
        prev_dones = torch.stack(prev_dones)
        log_probs, values = torch.stack(log_probs), torch.stack(values)
        next_values = torch.stack(next_values)
        hx = hx[0].clone()
        advantages = self.calculate_advantage(np.asarray(rewards), np.asarray(terms),
                                              np.asarray(truncs), values, next_values)
        returns = values + advantages
        stream = torch.cuda.current_stream(self.device).cuda_stream
        world, _ = dist_world()
        if cfg.advantage_norm:
            ms = torch.empty(4, dtype=torch.float32, device=self.device)
            if world > 1:
                # global statistics: this rank's {sum, sum^2}, all-reduced, then finalised
                sums = torch.empty(2, dtype=torch.float64, device=self.device)
                N.check(lib.dppo_adv_sums(h, sums.data_ptr(), stream), "dppo_adv_sums")
                torch.distributed.all_reduce(sums)
                n_total = float(cfg.rollout_steps * cfg.num_envs * world)
                N.check(lib.dppo_adv_stats_from_sums(sums.data_ptr(), n_total, ms.data_ptr(),
                                                     stream), "dppo_adv_stats_from_sums")
            else:
                N.check(lib.dppo_adv_stats(h, ms.data_ptr(), stream), "dppo_adv_stats")
            advantages = advantages.contiguous()
            N.check(lib.dppo_adv_normalize_f32(advantages.data_ptr(), ms.data_ptr(),
                                               advantages.numel(), stream), "normalize")
        flatten = lambda x: x.reshape(-1, *x.shape[2:])
        log_probs, actions, advantages, returns = [flatten(x) for x in
                                                   (log_probs, actions, advantages, returns)]
        B = cfg.rollout_steps * cfg.num_envs
        mb = B // cfg.num_minibatches
        perms = np.empty(cfg.num_epochs * B, np.int32)
        N.numpy_rng_permutations(B, cfg.num_epochs, perms)
        idx = torch.from_numpy(perms.astype(np.int64)).to(self.device).view(
            cfg.num_epochs, cfg.num_minibatches, mb)
        step = adam_step_count(self.optimizer, self.flat)
        lr = self.optimizer.param_groups[0]["lr"]
        if self.fused_gru and self.gru is not None:
            self._learn_fused(observations, actions, log_probs, advantages, returns, prev_dones,
                              hx, idx, step, lr, world, stream)
            advance_adam_steps(self.optimizer, self.flat, cfg.num_epochs * cfg.num_minibatches)
            self.lr_scheduler.step()
            return
        for b_idx in idx:
            for mb_idx in b_idx:
                self.flat.grad.zero_()
                nl, nv, _ = self.network.get_logits_values_and_hx(observations, hx, prev_dones)
                nl, nv = flatten(nl)[mb_idx], flatten(nv)[mb_idx]
                dist = torch.distributions.Categorical(logits=nl)
                ratio = (dist.log_prob(actions[mb_idx]) - log_probs[mb_idx]).exp()
                a = advantages[mb_idx]
                l_pi = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - cfg.ppo_clip,
                                                              1 + cfg.ppo_clip)).mean()
                l_v = 0.5 * torch.nn.functional.mse_loss(nv, returns[mb_idx])
                loss = l_pi + cfg.value_loss_weight * l_v - cfg.entropy_beta * dist.entropy().mean()
                if world > 1:
                    # local mean x 1/world, summed over the ranks = the union minibatch's mean
                    loss = loss * (1.0 / world)
                loss.backward()
                if world > 1:
                    torch.distributed.all_reduce(self.flat.grad)
                step += 1
                N.check(lib.dppo_clip_adam_f32(
                    self.flat.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                    self.v.data_ptr(), self.flat.total, cfg.grad_norm_clip, float(lr), 0.9, 0.999,
                    cfg.adam_eps, step, None, stream), "dppo_clip_adam_f32")
        advance_adam_steps(self.optimizer, self.flat, cfg.num_epochs * cfg.num_minibatches)
        self.lr_scheduler.step()

    def _learn_fused(self, observations, actions, log_probs, advantages, returns, prev_dones,
                     hx, idx, step, lr, world, stream):
        """Every minibatch: one dppo_gru_minibatch_grad_f32 launch (sequence recompute from hx,
        loss on the minibatch, BPTT; recurrent_ppo.py:335-360) -> [all-reduce] -> clip + Adam."""
        cfg, lib = self.cfg, self.gru.lib
        f32 = lambda x: x.to(torch.float32).contiguous()
        obs = f32(observations)
        act = actions.to(torch.int32).contiguous()
        old_lp, adv, ret = f32(log_probs), f32(advantages), f32(returns)
        dones = prev_dones.to(torch.uint8).contiguous()
        hx0 = f32(hx.reshape(cfg.num_envs, cfg.gru_hidden_dim))
        batch = N.GruBatch(obs.data_ptr(), act.data_ptr(), old_lp.data_ptr(), adv.data_ptr(),
                           ret.data_ptr(), dones.data_ptr(), hx0.data_ptr())
        hp = N.HParams(gamma=cfg.gamma, gae_lambda=cfg.gae_lambda, ppo_clip=cfg.ppo_clip,
                       value_loss_weight=cfg.value_loss_weight, entropy_beta=cfg.entropy_beta,
                       grad_norm_clip=cfg.grad_norm_clip, adam_beta1=0.9, adam_beta2=0.999,
                       adam_eps=cfg.adam_eps, advantage_norm=int(bool(cfg.advantage_norm)),
                       lr=float(lr), adam_step=int(step))
        idx32 = idx.to(torch.int32).contiguous()
        mb = idx32.shape[-1]
        m_total = mb * world          # the union minibatch's size under data parallelism
        total = self.flat.total
        losses = []
        for e in range(idx32.shape[0]):
            for j in range(idx32.shape[1]):
                mb_idx = idx32[e, j]
                N.check(lib.dppo_gru_minibatch_grad_f32(
                    self.gru.h, self.flat.flat.data_ptr(), ctypes.byref(batch), mb_idx.data_ptr(),
                    mb, m_total, ctypes.byref(hp), self.flat.grad.data_ptr(), stream),
                    "dppo_gru_minibatch_grad_f32")
                if world > 1:
                    torch.distributed.all_reduce(self.flat.grad)
                losses.append(self.flat.grad[total:total + 3].clone())
                step += 1
                N.check(lib.dppo_clip_adam_f32(
                    self.flat.flat.data_ptr(), self.flat.grad.data_ptr(), self.m.data_ptr(),
                    self.v.data_ptr(), total, cfg.grad_norm_clip, float(lr), 0.9, 0.999,
                    cfg.adam_eps, step, None, stream), "dppo_clip_adam_f32")
        # {loss, policy, value, entropy} per minibatch (reference never logs these; for tests)
        sums = torch.stack(losses) / float(m_total)
        self.last_losses = torch.stack([sums[:, 0] + cfg.value_loss_weight * sums[:, 1]
                                        - cfg.entropy_beta * sums[:, 2], sums[:, 0], sums[:, 1],
                                        sums[:, 2]], dim=1)

    def train(self) -> None:
        world, rank = dist_world()   # per-rank env seeds, rank-0 checkpoints (as PPO.train)
        seed = self.cfg.seed
        if seed is not None and world > 1:
            seed = seed + rank * self.cfg.num_envs
        self.current_observations, _ = self.envs.reset(seed=seed)
        self.prev_dones = np.zeros(self.cfg.num_envs, dtype=bool)
        self.current_hx = torch.zeros(1, self.cfg.num_envs, self.cfg.gru_hidden_dim,
                                      device=self.device)
        last = time.time()
        total = self.cfg.total_steps // (self.cfg.rollout_steps * self.cfg.num_envs)
        env_steps = 0
        for i in range(total):
            self.learn(self.rollout())
            env_steps = (i + 1) * self.cfg.rollout_steps * self.cfg.num_envs
            if self.cfg.checkpoint and rank == 0 and time.time() - last >= self.cfg.save_interval:
                self.checkpointer.save(env_steps, self.network, self.optimizer)
                last = time.time()
        if self.cfg.checkpoint and rank == 0:
            self.checkpointer.save(env_steps, self.network, self.optimizer)
        self.envs.close()
