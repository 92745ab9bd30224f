"""Minimal in-process stand-in for the `gymnasium` package (absent in this image).

Test infrastructure only.  Two users:

* ``make_golden.py`` injects it into ``sys.modules`` before importing the reference
  ``diamond`` package, which imports gymnasium unconditionally
  (reference ``diamond/ppo.py:6,10``) but only uses ``spaces.Box/Discrete`` type checks
  (``ppo.py:48-49``) and ``vector.SyncVectorEnv`` construction (``ppo.py:124-128``) on the
  learn() path.
* CPU tests of our own ``PPO.train()`` plumbing use the same synthetic env.

The fake vector env draws from its own ``numpy.random.default_rng`` so it never consumes the
global legacy NumPy RNG that drives the minibatch permutations (reference ``ppo.py:254``).
"""
from __future__ import annotations

import sys
import types

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = tuple(shape) if shape is not None else None
        self.dtype = dtype


class Box(Space):
    def __init__(self, low=-np.inf, high=np.inf, shape=None, dtype=np.float32):
        super().__init__(shape, dtype)
        self.low, self.high = low, high


class Discrete(Space):
    def __init__(self, n: int):
        super().__init__((), np.int64)
        self.n = int(n)


class SyntheticEnv:
    """One synthetic episodic env: Gaussian observations, N(1,1) rewards,
    termination w.p. p_term, truncation w.p. p_trunc per step."""

    def __init__(self, obs_dim=4, n_actions=2, continuous=False, act_dim=1,
                 p_term=0.02, p_trunc=0.005):
        self.observation_space = Box(shape=(obs_dim,))
        self.action_space = Box(shape=(act_dim,)) if continuous else Discrete(n_actions)
        self.p_term, self.p_trunc = p_term, p_trunc


class SyncVectorEnv:
    def __init__(self, env_fns, copy=True, autoreset_mode=None):
        self.envs = [fn() for fn in env_fns]
        self.num_envs = len(self.envs)
        e0 = self.envs[0]
        self.single_observation_space = e0.observation_space
        self.single_action_space = e0.action_space
        self._rng = np.random.default_rng(1234)
        self._d = int(np.prod(e0.observation_space.shape))

    def _obs(self, n):
        return self._rng.standard_normal((n, self._d)).astype(np.float32)

    def reset(self, seed=None, options=None):
        if seed is not None:
            self._rng = np.random.default_rng(seed)
        if options and "reset_mask" in options:
            mask = np.asarray(options["reset_mask"], dtype=bool)
            obs = self._last.copy()
            obs[mask] = self._obs(int(mask.sum()))
            self._last = obs
            return obs, {}
        self._last = self._obs(self.num_envs)
        return self._last, {}

    def step(self, actions):
        n = self.num_envs
        e0 = self.envs[0]
        obs = self._obs(n)
        rew = self._rng.normal(1.0, 1.0, n)
        term = self._rng.random(n) < e0.p_term
        trunc = self._rng.random(n) < e0.p_trunc
        self._last = obs
        return obs, rew, term, trunc, {}

    def close(self):
        pass


def install() -> None:
    """Register the stub as `gymnasium`, `gymnasium.spaces`, `gymnasium.vector`."""
    if "gymnasium" in sys.modules and getattr(sys.modules["gymnasium"], "_is_stub", False):
        return
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")
    vector = types.ModuleType("gymnasium.vector")
    spaces.Space, spaces.Box, spaces.Discrete = Space, Box, Discrete
    vector.SyncVectorEnv = SyncVectorEnv
    gym.spaces, gym.vector, gym.Env = spaces, vector, object
    gym._is_stub = True
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces,
                        "gymnasium.vector": vector})
