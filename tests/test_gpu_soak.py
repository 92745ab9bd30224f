"""Soak at the bench's production sizes: many back-to-back ``learn()`` calls of the fused HIP path
(old-policy eval, GAE, E x M minibatch kernels each followed by the optimizer step with its
grid-wide tagged-word fan-in, look-ahead permutation drafts), run twice from the same state.

The two runs must end bit-identical -- parameters and the last learn's per-minibatch trace
(losses, grad norms) -- and the handle's sticky device error word must stay clear.  This is the
check for what a single learn cannot show: a fan-in whose launch epochs wrap or go stale, a
draft consumed out of order, a tag word read before it is published, an accumulation that
depends on timing.  The numerics of one learn against the oracle are test_gpu_production.py's;
the trace's determinism over 1-2 learns, test_gpu_parity.py's.  Configurations: bench.py's C2 /
C3 / C4 and C5 on one GPU (reference ppo.py:224-287, continuous_ppo.py:236-299)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import bench
import diamond


def _soak(name: str, learns: int, seed: int):
    model, T, Nc, D, A, cont, pt, ptr, _ = bench.CONFIGS[name]
    np.random.seed(seed)
    torch.manual_seed(seed)
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=Nc, verbose=False, total_steps=10 ** 12)
    agent = Agent(None, cfg, envs=bench.SpecEnvs(D, A, cont))
    L = agent._learner
    assert L.fused, "the soak must run the fused HIP path"
    dev = torch.device("cuda:0")
    ro, _ = bench.synth_rollout(T, Nc, D, A, cont, pt, ptr, seed=seed, device=dev)
    before = np.concatenate([p.detach().cpu().numpy().ravel() for p in agent.network.parameters()])
    for _ in range(learns):
        agent.learn_device(ro)
    torch.cuda.synchronize(dev)
    status = L.handle.lib.dppo_status(L.handle.h)
    trace = L.handle.trace(cfg.num_epochs * cfg.num_minibatches)
    after = np.concatenate([p.detach().cpu().numpy().ravel() for p in agent.network.parameters()])
    agent.close()
    return status, before, after, trace


@pytest.mark.timeout(240)
@pytest.mark.parametrize("name,learns", [("cartpole4096", 300), ("lunar8192", 200),
                                         ("cheetah4096", 300), ("c5", 40)])
def test_back_to_back_learns_are_bit_identical_and_error_free(name, learns):
    s1, b1, a1, t1 = _soak(name, learns, seed=5)
    s2, b2, a2, t2 = _soak(name, learns, seed=5)
    assert s1 == 0 and s2 == 0, (s1, s2)                  # no fan-in / tag timeout raised
    assert np.array_equal(b1, b2)                        # same initial network
    assert np.isfinite(a1).all() and np.isfinite(t1).all()
    assert not np.array_equal(a1, b1)                    # the learns did update the network
    assert np.array_equal(a1, a2), f"{name}: parameters differ after {learns} learns"
    assert np.array_equal(t1, t2), f"{name}: last learn's trace differs"
