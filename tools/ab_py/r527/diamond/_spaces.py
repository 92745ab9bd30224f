"""Space checks and the vector-env constructor, with gymnasium imported lazily.

The reference imports gymnasium unconditionally (diamond/ppo.py:6,10) but the hot path only uses
``spaces.Box`` / ``spaces.Discrete`` type checks (ppo.py:48-49) and ``vector.SyncVectorEnv``
(ppo.py:124-128).  gymnasium is not part of this image, so the learn() path must not need it;
when it is installed the real classes are used.
"""
from __future__ import annotations


def _gym():
    try:
        import gymnasium  # noqa: F401
        return gymnasium
    except ImportError:
        return None


def is_box(space) -> bool:
    g = _gym()
    if g is not None and isinstance(space, g.spaces.Space):
        return isinstance(space, g.spaces.Box)
    return type(space).__name__ == "Box" and getattr(space, "shape", None) is not None


def is_discrete(space) -> bool:
    g = _gym()
    if g is not None and isinstance(space, g.spaces.Space):
        return isinstance(space, g.spaces.Discrete)
    return type(space).__name__ == "Discrete" and hasattr(space, "n")


def make_vector_env(env_fn, num_envs: int):
    """gym.vector.SyncVectorEnv([...], copy=True, autoreset_mode="Disabled")  (ppo.py:124-128)."""
    g = _gym()
    if g is None:
        raise ImportError("gymnasium is required to construct environments (rollout/train); "
                          "learn() on staged buffers does not need it")
    return g.vector.SyncVectorEnv([env_fn for _ in range(num_envs)], copy=True,
                                  autoreset_mode="Disabled")
