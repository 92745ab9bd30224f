"""diamond -- MI355X (gfx950) native PPO hot path, drop-in for Auxeno/diamond-ppo.

Exports the reference's six names (reference diamond/__init__.py:1-3).  Everything heavy runs in
libdppo.so (HIP kernels + C ABI, include/dppo.h); this package is the host-side mirror of the
reference's classes around it.
"""
from .ppo import PPO, PPOConfig
from .recurrent_ppo import RecurrentPPO, RecurrentPPOConfig
from .continuous_ppo import ContinuousPPO, ContinuousPPOConfig

__all__ = ["PPO", "PPOConfig", "RecurrentPPO", "RecurrentPPOConfig", "ContinuousPPO",
           "ContinuousPPOConfig"]
