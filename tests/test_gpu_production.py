"""GPU parity of the minibatch kernels in their PRODUCTION configuration.

Two kernels compute a minibatch gradient (csrc/common.h launch_mb):
* the sample-split kernel (csrc/mbwave.hip; <= 4 actions, <= 8 discrete on <= 16 inputs, or
  HalfCheetah's 5-6 Gaussian actions on exactly 17 inputs -- the X1 instantiation):
  G = min(ceil(m/64), 256) workgroups of 4 waves, each wave running ceil(ceil(m/16) / 4G)
  16-sample groups end to end and accumulating its own weight gradients across them (C2: 4
  groups per wave, C3: 8).  The golden-trace tests have minibatches of at most 4,096 samples, i.e.
  one group per wave: the cross-group accumulation and prefetch are first exercised here;
* the two-team kernel (csrc/mbstep.hip; the other 5-8-action shapes, e.g. 6 Gaussian actions on
  20 inputs; HalfCheetah too under DPPO_MBW_CONT6=0):
  G = min(ceil(m/32), 256) workgroups, each running nit = ceil(ceil(m/32)/G) 32-sample steps
  through a two-team software pipeline (the forward team on step it while the backward team
  back-propagates step it-1, hand-off images double-buffered by step parity); small minibatches
  have nit == 1 and never read the odd-parity buffers.
These tests run the production shapes:

* one minibatch gradient at the full C2 / C3 / C4 minibatch sizes (65,536 / 131,072 / 65,536
  samples: 4 / 8 / 4 groups per wave), plus a ragged one (m % 32 != 0, workgroups with unequal step
  counts), through ``dppo_minibatch_grad_f32`` against the oracle's ``minibatch_loss_grads`` on the
  same sample records and indices (reference ppo.py:261-283, continuous_ppo.py:273-295);
* one minibatch gradient at C5's one-GPU size (1,048,576 samples: 64 groups per wave);
* a full ``learn()`` at intermediate sizes (depth 1-3, both kernels, discrete and continuous) and at the full
  C2, C3 and C4 sizes (4 / 8 / 4 groups per wave) against the oracle's ``learn`` with the same
  NumPy permutations (ppo.py:224-287, continuous_ppo.py:236-299).

Tolerances.  At these sizes every gradient entry is a sum of 65,536-131,072 fp32 terms, so BOTH
fp32 implementations (the kernel and the NumPy oracle) carry a summation error of order
eps32 * sqrt(m) relative to max|g| (~1.5e-5 at m = 65,536).  The yardstick is therefore the same
oracle evaluated in float64 (``dt=np.float64``): the kernel must be within 2e-5 * max|g| of it
per entry -- the small-size golden-trace bound -- and no further from it than 4x the fp32
oracle's own distance (+1e-6 * max|g|).  Full learn(): losses / grad norms rel 1e-4 and
parameters 2e-5 abs after 32 Adam steps against the fp32 oracle (test_learn_large_vs_oracle's
bounds).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import diamond
from diamond import _native as N
from oracle import ppo_np as P

from gpu_helpers import (H, SpecEnvs, dev, hparams, production_depth, random_params, stream,
                         synth)


# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,T,Nn,D,A,cont,ragged", [
    ("C2 cartpole", 128, 4096, 4, 2, False, 0),
    ("C3 lunar", 128, 8192, 8, 4, False, 0),
    ("C4 cheetah", 128, 4096, 17, 6, True, 0),
    ("C2 ragged", 128, 4096, 4, 2, False, 77),
    ("C4 ragged", 128, 4096, 17, 6, True, 4093),
    # BASELINE configs[4] on ONE GPU (bench configs_extra.c5): 1,048,576-sample minibatches, 64
    # groups per wave accumulated in the wave's registers
    ("C5 one GPU", 128, 65536, 4, 2, False, 0),
    ("7 discrete actions", 128, 4096, 6, 7, False, 0),
    ("3 Gaussian actions, 20 inputs", 128, 4096, 20, 3, True, 13),
])
def test_full_minibatch_gradient_vs_oracle(name, T, Nn, D, A, cont, ragged):
    E, M = 4, 8
    B = T * Nn
    h = N.Handle(0, N.Dims(T, Nn, D, A, int(cont), H, E, M, 1, 0))
    L = h.layout
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    rng = np.random.default_rng(B + D)
    params, flat = random_params(L, names, D, A, cont, rng)
    ro, host = synth(T, Nn, D, A, cont, seed=D * 7 + A)
    pd = torch.from_numpy(flat).to(dev())
    outs = {k: torch.empty(B, device=dev()) for k in
            ("log_probs", "values", "next_values", "advantages", "returns")}
    lo = N.LearnOutputs(*[outs[k].data_ptr() for k in
                          ("log_probs", "values", "next_values", "advantages", "returns")])
    hp = hparams()
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), pd.data_ptr(),
                                   ctypes.byref(hp), ctypes.byref(lo), stream()))
    mb = B // M - ragged
    assert production_depth(mb, D, A, cont) >= 4
    idx = np.random.RandomState(B).permutation(B)[:mb].astype(np.int32)
    idx_d = torch.from_numpy(idx).to(dev())
    g = torch.zeros(L.total, device=dev())
    loss4 = (ctypes.c_float * 4)()
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, pd.data_ptr(), idx_d.data_ptr(), mb, mb,
                                          ctypes.byref(hp), g.data_ptr(), loss4, stream()))
    torch.cuda.synchronize()
    got_flat = g.cpu().numpy()
    got = np.concatenate([got_flat[L.offset[i]:L.offset[i] + L.numel[i]] for i in range(L.count)])
    o = {k: v.cpu().numpy() for k, v in outs.items()}
    obs, _, act, *_ = host
    obs_f = obs.reshape(B, D)
    act_f = act.reshape(B, A) if cont else act.reshape(B)
    args = (obs_f[idx], act_f[idx], o["log_probs"][idx], o["advantages"][idx], o["returns"][idx])
    res = {}
    for dt in (np.float32, np.float64):
        loss, comps, grads = P.minibatch_loss_grads(params, *args, P.Hyper(), cont, dt=dt)
        res[dt] = (loss, comps, np.concatenate([np.asarray(grads[n], np.float64).ravel()
                                                for n in names]))
    exact = res[np.float64][2]
    scale = np.abs(exact).max()
    err_kernel = np.abs(got - exact).max() / scale
    err_oracle32 = np.abs(res[np.float32][2] - exact).max() / scale
    assert err_kernel <= 2e-5, (name, err_kernel, err_oracle32)
    assert err_kernel <= 4 * err_oracle32 + 1e-6, (name, err_kernel, err_oracle32)
    # per tensor, relative to the tensor's own scale (small tensors are not hidden by big ones)
    for i, n in enumerate(names):
        a = got[sum(L.numel[k] for k in range(i)):][:L.numel[i]]
        b = exact[sum(L.numel[k] for k in range(i)):][:L.numel[i]]
        s = max(np.abs(b).max(), 1e-3 * scale)
        assert np.abs(a - b).max() <= 1e-4 * s, (name, n, np.abs(a - b).max() / s)
    loss, comps, _ = res[np.float64]
    assert abs(loss4[0] - loss) <= 2e-5 * max(1.0, abs(loss)), (loss4[0], loss)
    assert abs(loss4[1] - comps["loss_policy"]) <= 2e-5 * max(1.0, abs(comps["loss_policy"]))
    assert abs(loss4[2] - comps["loss_value"]) <= 2e-5 * max(1.0, abs(comps["loss_value"]))
    assert abs(loss4[3] - comps["entropy"]) <= 2e-5 * max(1.0, abs(comps["entropy"]))


@pytest.mark.parametrize("name,T,Nn,D,A,cont", [
    ("C3 lunar eval", 128, 8192, 8, 4, False),
    ("C4 cheetah eval", 128, 4096, 17, 6, True),
])
def test_full_size_old_policy_and_records_vs_oracle(name, T, Nn, D, A, cont):
    """prepare() at full BASELINE sizes: old-policy log-probs / values / next-values (eval_kernel)
    against the oracle's old_policy, advantages bit-exact through GAE, normalisation rel 2e-6."""
    E, M = 4, 8
    B = T * Nn
    h = N.Handle(0, N.Dims(T, Nn, D, A, int(cont), H, E, M, 1, 0))
    L = h.layout
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    params, flat = random_params(L, names, D, A, cont, np.random.default_rng(3))
    ro, host = synth(T, Nn, D, A, cont, seed=11)
    pd = torch.from_numpy(flat).to(dev())
    outs = {k: torch.empty(B, device=dev()) for k in
            ("log_probs", "values", "next_values", "advantages", "returns")}
    lo = N.LearnOutputs(*[outs[k].data_ptr() for k in
                          ("log_probs", "values", "next_values", "advantages", "returns")])
    hp = hparams()
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), pd.data_ptr(),
                                   ctypes.byref(hp), ctypes.byref(lo), stream()))
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in outs.items()}
    obs, nobs, act, rew, te, tr = host
    logp, v, nv, _ = P.old_policy(params, obs, act, nobs, cont)
    np.testing.assert_allclose(o["log_probs"], logp.ravel(), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["values"], v.ravel(), rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["next_values"], nv.ravel(), rtol=2e-5, atol=2e-5)
    # GAE on the kernel's own values is bit-exact; the stored returns are values + raw advantages
    vals = o["values"].reshape(T, Nn)
    adv = P.gae(rew, te, tr, vals, o["next_values"].reshape(T, Nn))
    assert np.array_equal(o["returns"].reshape(T, Nn), vals + adv)
    np.testing.assert_allclose(o["advantages"], P.normalize_adv(adv).ravel(), rtol=0, atol=2e-6)


# ---------------------------------------------------------------------------------------------
def learn_vs_oracle(T, Nn, D, A, cont, seed):
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=Nn, verbose=False)
    agent = Agent(None, cfg, envs=SpecEnvs(D, A, cont))
    assert agent._learner.fused
    mb = T * Nn // cfg.num_minibatches
    names = [n for n, _ in agent.network.named_parameters()]
    params = {n: p.detach().cpu().numpy().copy() for n, p in agent.network.named_parameters()}
    ro, host = synth(T, Nn, D, A, cont, seed)
    np.random.seed(seed)
    st = np.random.get_state()
    agent.learn_device(ro)
    tr = agent.learn_trace()
    torch.cuda.synchronize()
    np.random.set_state(st)
    adam = P.new_adam_state(params, names)
    ref = P.learn(params, adam, list(host), P.Hyper(), cfg.lr, cont, rng=np.random)
    np.testing.assert_allclose(tr[:, 0], ref["loss"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(tr[:, 4], ref["norm"], rtol=1e-4, atol=1e-5)
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), params[n], rtol=0, atol=2e-5,
                                   err_msg=n)
    return mb


@pytest.mark.parametrize("T,Nn,D,A,cont,want_depth", [
    (128, 2048, 4, 2, False, 2),     # sample-split, mb 32,768: two groups per wave
    (128, 1536, 8, 4, False, 2),     # 1,536 groups over 1,024 waves: some waves two, some one
    (100, 3000, 5, 3, False, 3),     # mb 37,500: three groups per wave, the last group partial
    (100, 1000, 5, 3, False, 1),     # mb 12,500: 196 workgroups, the last group partial
    (128, 2048, 3, 1, True, 2),      # Gaussian head on the sample-split kernel
    (128, 1536, 17, 6, True, 2),     # HalfCheetah's X1 sample-split kernel: some waves two groups
    (128, 768, 20, 6, True, 2),      # two-team kernel: 384 steps over 256 workgroups (ragged nit)
])
def test_learn_intermediate_depth_vs_oracle(T, Nn, D, A, cont, want_depth):
    mb = learn_vs_oracle(T, Nn, D, A, cont, seed=T + Nn)
    assert production_depth(mb, D, A, cont) == want_depth


@pytest.mark.parametrize("cont", [False, True])
def test_learn_at_the_shape_limits_vs_oracle(cont):
    """The C-ABI's largest MLP shape, 32 inputs and 16 actions (the two-team kernel's 16-head
    build, the 16-head eval and the widest sample records): the 32-step learn() against the
    oracle's."""
    learn_vs_oracle(16, 256, 32, 16, cont, seed=16 + cont)


def test_learn_full_c2_vs_oracle():
    """BASELINE configs[1] itself: CartPole PPO, T = 128, N = 4096 (mb 65,536: four groups per
    wave of the sample-split kernel)."""
    mb = learn_vs_oracle(128, 4096, 4, 2, False, seed=0)
    assert production_depth(mb, 4, 2, False) == 4


def test_learn_full_c3_vs_oracle():
    """BASELINE configs[2], the bench headline: LunarLander PPO, T = 128, N = 8192 (mb 131,072:
    eight groups per wave of the sample-split kernel), the full 32-step learn() against the
    oracle's learn with the same NumPy permutations (ppo.py:224-287)."""
    mb = learn_vs_oracle(128, 8192, 8, 4, False, seed=2)
    assert production_depth(mb, 8, 4, False) == 8


def test_learn_full_c4_vs_oracle():
    """BASELINE configs[3]: HalfCheetah ContinuousPPO, T = 128, N = 4096 (mb 65,536: four groups
    per wave of the X1 sample-split instantiation), the full 32-step learn() against the oracle's
    learn (continuous_ppo.py:236-299)."""
    mb = learn_vs_oracle(128, 4096, 17, 6, True, seed=3)
    assert production_depth(mb, 17, 6, True) == 4


# ---------------------------------------------------------------------------------------------
def test_grid_fanin_reports_non_resident_grid():
    """The single-device optimizer step (reduce_adam_kernel, and the optional fused tail of the
    minibatch kernel) meets in a grid-wide fan-in.  Its wait is bounded: a grid that cannot be
    co-resident drains after the timeout and raises the handle's sticky error, which every later
    call reports (DPPO_EHIP -> RuntimeError) -- an error return, not numbers from stale partials."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    T, Nn, D, A = 16, 64, 4, 2
    h = N.Handle(0, N.Dims(T, Nn, D, A, 0, H, 4, 8, 1, 0))
    lib = h.lib
    # resident: one 1024-thread workgroup per CU (96 KB of LDS each: two never share a CU)
    N.check(lib.dppo_fanin_selftest(h.h, cus, 96 * 1024, 2_000_000, stream()))
    torch.cuda.synchronize()
    assert lib.dppo_status(h.h) == N.DPPO_OK
    # a learn on the same handle still works and moves the parameters
    L = h.layout
    names = P.DISCRETE_NAMES
    params, flat = random_params(L, names, D, A, False, np.random.default_rng(0))
    ro, _ = synth(T, Nn, D, A, False, seed=1)
    pd = torch.from_numpy(flat).to(dev())
    m = torch.zeros_like(pd)
    v = torch.zeros_like(pd)
    perms = np.stack([np.random.RandomState(e).permutation(T * Nn) for e in range(4)]).astype(np.int32)
    hp = hparams()
    st = ro.as_struct()
    N.check(lib.dppo_learn_f32(h.h, ctypes.byref(st), pd.data_ptr(), m.data_ptr(), v.data_ptr(),
                               ctypes.byref(hp), perms.ctypes.data, None, stream()))
    torch.cuda.synchronize()
    after_ok = pd.cpu().numpy()
    assert not np.array_equal(after_ok, flat)
    # NOT co-resident: 8 more workgroups than CUs, each needing a CU of its own
    N.check(lib.dppo_fanin_selftest(h.h, cus + 8, 96 * 1024, 20_000, stream()))
    torch.cuda.synchronize()
    assert lib.dppo_status(h.h) == N.DPPO_EHIP
    msg = lib.dppo_last_error().decode()
    assert "fan-in timed out" in msg
    # the error word names the first wait that gave up: code 1, the workgroup that raised it
    import re
    hit = re.search(r"code 1, block (\d+)", msg)
    assert hit and int(hit.group(1)) < cus + 8, msg
    rc = lib.dppo_learn_f32(h.h, ctypes.byref(st), pd.data_ptr(), m.data_ptr(), v.data_ptr(),
                            ctypes.byref(hp), perms.ctypes.data, None, stream())
    assert rc == N.DPPO_EHIP
    torch.cuda.synchronize()
    assert np.array_equal(pd.cpu().numpy(), after_ok)   # nothing was enqueued
    with pytest.raises(N.NativeError):
        h.trace(32)
