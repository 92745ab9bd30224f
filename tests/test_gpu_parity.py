"""GPU parity tests: the HIP path (through the C ABI / the drop-in classes) against the golden
fixtures captured from the reference and against the CPU oracle.

Tolerances (SURVEY.md §7.2 hard part 2):
* GAE advantages and returns: bit-exact (reference fp32 op order, no FMA contraction).
* old-policy log-probs / values: |diff| <= 2e-5 (fp32 MLP, different GEMM summation order).
* gradients: max|diff| <= 2e-5 x max|g| per step; losses / grad norms: rel 2e-5.
* parameters after every Adam step: |diff| <= 5e-6 (Adam's first steps are ~lr*sign(g)).
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import LEARN_TRACES, load_golden

pytestmark = pytest.mark.gpu

import diamond
from diamond import _native as N
from diamond.engine import DeviceRollout


def dev():
    return torch.device("cuda", 0)


def t(x, dtype=None):
    a = torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None:
        a = a.to(dtype)
    return a.to(dev()).contiguous()


def stream():
    return torch.cuda.current_stream().cuda_stream


def gae_handle(T, Nn):
    return N.Handle(0, N.Dims(T, Nn, 1, 1, 0, 64, 1, 1, 1, 0))


# ---------------------------------------------------------------------------------------------
def run_gae(r, te, tr, v, nv, mode=0):
    T, Nn = r.shape
    h = gae_handle(T, Nn)
    h.set_gae_mode(mode)
    adv = torch.empty(T, Nn, device=dev())
    ret = torch.empty(T, Nn, device=dev())
    ms = torch.zeros(4, device=dev())
    args = [t(r, torch.float32), t(te, torch.uint8), t(tr, torch.uint8), t(v, torch.float32),
            t(nv, torch.float32)]
    N.check(h.lib.dppo_gae_f32(h.h, *[a.data_ptr() for a in args], adv.data_ptr(), ret.data_ptr(),
                               0.99, 0.95, stream()))
    N.check(h.lib.dppo_adv_stats(h.h, ms.data_ptr(), stream()))
    norm = adv.clone()
    N.check(h.lib.dppo_adv_normalize_f32(norm.data_ptr(), ms.data_ptr(), norm.numel(), stream()))
    torch.cuda.synchronize()
    return adv.cpu().numpy(), ret.cpu().numpy(), ms.cpu().numpy(), norm.cpu().numpy()


def test_gae_bitexact_golden():
    d = load_golden("gae_cases.npz")
    for n in d["names"]:
        adv, ret, ms, norm = run_gae(d[n + "/rewards"], d[n + "/term"], d[n + "/trunc"],
                                     d[n + "/values"], d[n + "/next_values"])
        assert np.array_equal(adv, d[n + "/adv"]), n
        assert np.array_equal(ret, d[n + "/returns"]), n
        if adv.size > 1:
            assert abs(ms[0] - d[n + "/mean"]) <= 1e-6 * max(1.0, abs(float(d[n + "/mean"]))), n
            assert abs(ms[1] - d[n + "/std"]) <= 1e-6 * float(d[n + "/std"]), n
            np.testing.assert_allclose(norm, d[n + "/adv_norm"], rtol=0, atol=2e-6, err_msg=n)


@pytest.mark.parametrize("T,Nn", [(128, 8192), (128, 4096), (300, 16), (1, 1), (129, 33),
                                  (7, 4104), (200, 8448), (64, 6144), (16, 12288),
                                  (128, 65536), (200, 16384), (64, 16448)])
def test_gae_vs_oracle_sizes(T, Nn):
    from oracle import ppo_np as P
    rng = np.random.default_rng(T * 31 + Nn)
    r = rng.normal(1, 1, (T, Nn)).astype(np.float32)
    te = (rng.random((T, Nn)) < 0.02).astype(np.uint8)
    tr = (rng.random((T, Nn)) < 0.005).astype(np.uint8)
    v = rng.standard_normal((T, Nn)).astype(np.float32)
    nv = rng.standard_normal((T, Nn)).astype(np.float32)
    adv, ret, ms, _ = run_gae(r, te, tr, v, nv)
    ref = P.gae(r, te, tr, v, nv)
    assert np.array_equal(adv, ref)
    assert np.array_equal(ret, v + ref)
    if adv.size > 1:
        mean, std = P.adv_stats(ref)
        assert abs(ms[0] - mean) <= 1e-6 * max(1.0, abs(mean))
        assert abs(ms[1] - std) <= 2e-6 * std


@pytest.mark.parametrize("T,Nn,mode", [(128, 8192, 0), (128, 4096, 0), (128, 65536, 0),
                                       (129, 33, 0), (64, 6144, 0), (300, 64, 0),
                                       (128, 8192, 1), (128, 65536, 1)])
def test_gae_stats_large_mean(T, Nn, mode):
    """Normalisation statistics when the advantages' mean dwarfs their spread: every step terminal
    (adv = r - v), v = -1,000, r ~ N(0, 1), so mean / std ~ 1,000 -- the case in which fp32
    partial sums lose the variance (the kernels shift each lane's chunk by its first advantage).
    Mean and std within 1e-6 / 2e-6 of the float64 oracle (P.adv_stats), the normalised
    advantages within 2e-6 of P.normalize_adv; every kernel (32-, 16-, 64-env tiles, the
    unaligned serial kernel, super-chunks, and the affine mode)."""
    from oracle import ppo_np as P
    rng = np.random.default_rng(T * 7 + Nn)
    r = rng.standard_normal((T, Nn)).astype(np.float32)
    te = np.ones((T, Nn), np.uint8)
    tr = np.zeros((T, Nn), np.uint8)
    v = np.full((T, Nn), -1000.0, np.float32)
    nv = rng.standard_normal((T, Nn)).astype(np.float32)
    adv, ret, ms, norm = run_gae(r, te, tr, v, nv, mode=N.GAE_AFFINE if mode else 0)
    ref = P.gae(r, te, tr, v, nv)
    if not mode:
        assert np.array_equal(adv, ref)
    mean, std = P.adv_stats(ref)
    assert abs(ms[0] - mean) <= 1e-6 * abs(mean), (ms[0], mean)
    assert abs(ms[1] - std) <= 2e-6 * std, (ms[1], std)
    np.testing.assert_allclose(norm, P.normalize_adv(adv), rtol=0, atol=2e-6)


@pytest.mark.parametrize("T,Nn", [(128, 8192), (128, 65536), (128, 4096), (300, 64),
                                  (129, 4096), (200, 8448), (64, 6144), (16, 12288), (1, 32),
                                  (100, 512), (7, 4104)])
def test_gae_affine_mode_within_tolerance(T, Nn):
    """DPPO_GAE_AFFINE (SURVEY §7.2 / §8(c) tolerance mode): every chunk's affine map composed in
    parallel.  Against the bit-exact oracle: |adv - ref| <= 1e-6 x max|ref| (and returns the
    same), statistics rel 1e-6; T > 128 chains super-chunks, T % 16 != 0 and T < 16 leave
    identity rows, N % 32 != 0 runs the 16-env tiles (N % 16 != 0: the serial kernel)."""
    from oracle import ppo_np as P
    rng = np.random.default_rng(T * 17 + Nn)
    r = rng.normal(1, 1, (T, Nn)).astype(np.float32)
    te = (rng.random((T, Nn)) < 0.02).astype(np.uint8)
    tr = (rng.random((T, Nn)) < 0.005).astype(np.uint8)
    v = rng.standard_normal((T, Nn)).astype(np.float32)
    nv = rng.standard_normal((T, Nn)).astype(np.float32)
    adv, ret, ms, _ = run_gae(r, te, tr, v, nv, mode=N.GAE_AFFINE)
    ref = P.gae(r, te, tr, v, nv)
    scale = float(np.abs(ref).max())
    err = np.abs(adv.astype(np.float64) - ref).max()
    assert err <= 1e-6 * scale, (err, scale)
    assert np.abs(ret.astype(np.float64) - (v + ref)).max() <= 1e-6 * scale + 1e-6
    if T % 16 == 0:  # the rollout's last 16 steps start from carry 0: bit-exact
        assert np.array_equal(adv[-16:], ref[-16:])
    mean, std = P.adv_stats(ref)
    assert abs(ms[0] - mean) <= 1e-6 * max(1.0, abs(mean))
    assert abs(ms[1] - std) <= 2e-6 * std


@pytest.mark.parametrize("name", ["lunar_medium", "cheetah_small", "cartpole_c1"])
def test_learn_with_affine_gae_matches_reference_trace(name):
    """learn() with the tolerance-mode GAE (cfg.gae_bitexact = False) stays within the golden
    traces' tolerances (advantages 5e-5, losses / norms rel 2e-5, parameters 5e-6)."""
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, n_learn = (int(x) for x in z["dims"])
    agent = make_agent(z)
    agent._learner.handle.set_gae_mode(N.GAE_AFFINE)
    losses = []
    for li in range(n_learn):
        np.random.set_state(("MT19937", z[f"rng_state_before{li}"].astype(np.uint32),
                             int(z[f"rng_pos_before{li}"]), 0, 0.0))
        ro = diamond.engine.stage_experience(experience(z, li), dev(), bool(cont))
        agent.learn_device(ro)
        losses += list(agent.learn_trace()[:, 0])
    torch.cuda.synchronize()
    np.testing.assert_allclose(losses, z["loss"], rtol=2e-5, atol=2e-5)
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0, atol=5e-6,
                                   err_msg=n)


def test_gae_full_size_properties():
    """BASELINE sizes, size-independent checks: no dones => discounted-sum identity; all
    terminated => adv = r - v."""
    T, Nn = 128, 8192
    rng = np.random.default_rng(5)
    r = rng.normal(1, 1, (T, Nn)).astype(np.float32)
    v = rng.standard_normal((T, Nn)).astype(np.float32)
    nv = rng.standard_normal((T, Nn)).astype(np.float32)
    z = np.zeros((T, Nn), np.uint8)
    o = np.ones((T, Nn), np.uint8)
    adv, _, _, _ = run_gae(r, o, z, v, nv)
    assert np.array_equal(adv, r - v)
    adv, _, _, _ = run_gae(r, z, z, v, nv)
    delta = r.astype(np.float64) + 0.99 * nv - v
    ref = np.zeros_like(delta)
    a = 0.0
    for k in range(T - 1, -1, -1):
        a = delta[k] + 0.99 * 0.95 * a
        ref[k] = a
    np.testing.assert_allclose(adv, ref, rtol=1e-4, atol=1e-4)


# ---------------------------------------------------------------------------------------------
def make_agent(z):
    import gym_stub
    T, Nn, D, A, cont, _ = (int(x) for x in z["dims"])
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    kw = {k: z["cfg/" + k].item() for k in ("num_epochs", "num_minibatches", "lr", "adam_eps",
                                             "gamma", "gae_lambda", "ppo_clip",
                                             "value_loss_weight", "entropy_beta",
                                             "grad_norm_clip", "total_steps")}
    cfg = Cfg(rollout_steps=T, num_envs=Nn, verbose=False,
              advantage_norm=bool(z["cfg/advantage_norm"]), decay_lr=bool(z["cfg/decay_lr"]), **kw)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A, continuous=bool(cont),
                                                                 act_dim=A)] * Nn)
    agent = Agent(None, cfg, envs=envs)
    sd = {n: torch.from_numpy(z["init/" + n]) for n in z["param_names"]}
    if hasattr(agent.network, "actor_out_layer"):  # alias of actor_head.2 in the state_dict
        sd["actor_out_layer.weight"] = sd["actor_head.2.weight"]
        sd["actor_out_layer.bias"] = sd["actor_head.2.bias"]
    agent.network.load_state_dict(sd)
    return agent


def experience(z, li):
    keys = ("obs", "next_obs", "actions", "rewards", "term", "trunc")
    arrs = [z[f"exp{li}/" + k] for k in keys]
    T = arrs[0].shape[0]
    return [[a[k] for a in arrs] for k in range(T)]


def flat_params(agent):
    return np.concatenate([p.detach().cpu().numpy().ravel() for p in agent.network.parameters()])


@pytest.mark.parametrize("name,device_shuffle,fused_adam",
                         [(n, False, False) for n in LEARN_TRACES] +
                         [("cartpole_decay", True, False), ("cheetah_small", True, False),
                          ("lunar_medium", False, True), ("cheetah_small", False, True),
                          ("cartpole_small", False, "split"), ("lunar_medium", False, "split"),
                          ("cheetah_small", False, "split"), ("pendulum_medium", False, "split")])
def test_learn_matches_reference_trace(name, device_shuffle, fused_adam, monkeypatch):
    """Full drop-in learn() through the fused HIP path vs the reference's captured trace,
    including the NumPy-RNG minibatch order (global RNG set to the captured state); also with the
    slab reduction + clip + Adam as the minibatch kernel's tail (DPPO_FUSED_ADAM=1), and with the
    multi-GPU per-minibatch sequence (minibatch kernel -> slab_reduce_kernel -> [RCCL] ->
    clip_adam_kernel) forced on one device (DPPO_SPLIT_ADAM=1)."""
    monkeypatch.delenv("DPPO_FUSED_ADAM", raising=False)
    monkeypatch.delenv("DPPO_SPLIT_ADAM", raising=False)
    if fused_adam == "split":
        monkeypatch.setenv("DPPO_SPLIT_ADAM", "1")
    elif fused_adam:
        monkeypatch.setenv("DPPO_FUSED_ADAM", "1")
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, n_learn = (int(x) for x in z["dims"])
    agent = make_agent(z)
    assert agent._learner.fused
    agent._learner.device_shuffle = device_shuffle
    E, M = int(z["cfg/num_epochs"]), int(z["cfg/num_minibatches"])
    losses, norms, params_after = [], [], []
    for li in range(n_learn):
        np.random.set_state(("MT19937", z[f"rng_state_before{li}"].astype(np.uint32),
                             int(z[f"rng_pos_before{li}"]), 0, 0.0))
        B = T * Nn
        outs = {k: torch.empty(B, device=dev()) for k in
                ("log_probs", "values", "next_values", "advantages", "returns")}
        lo = N.LearnOutputs(*[outs[k].data_ptr() for k in
                              ("log_probs", "values", "next_values", "advantages", "returns")])
        ro = diamond.engine.stage_experience(experience(z, li), dev(), bool(cont))
        agent.learn_device(ro, lo)
        tr = agent.learn_trace()
        losses += list(tr[:, 0])
        norms += list(tr[:, 4])
        torch.cuda.synchronize()
        np.testing.assert_allclose(outs["log_probs"].cpu().numpy(), z["old/log_probs"][li].ravel(),
                                   atol=2e-5, err_msg="old log_probs")
        np.testing.assert_allclose(outs["values"].cpu().numpy(), z["old/values"][li].ravel(),
                                   atol=2e-5, err_msg="values")
        np.testing.assert_allclose(outs["next_values"].cpu().numpy(),
                                   z["old/next_values"][li].ravel(), atol=2e-5, err_msg="next_values")
        np.testing.assert_allclose(outs["returns"].cpu().numpy() - outs["values"].cpu().numpy(),
                                   z["old/adv"][li].ravel(), atol=5e-5, err_msg="advantages")
        params_after.append(flat_params(agent))
        # the global NumPy RNG ends where the reference left it (state before the next learn)
        if li + 1 < n_learn:
            st = np.random.get_state()
            assert np.array_equal(st[1], z[f"rng_state_before{li + 1}"].astype(np.uint32))
            assert st[2] == int(z[f"rng_pos_before{li + 1}"])
    np.testing.assert_allclose(losses, z["loss"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(norms, z["norm"], rtol=2e-5, atol=2e-5)
    names = list(z["param_names"])
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0, atol=5e-6,
                                   err_msg=n)
        st = agent.optimizer.state[p]
        np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), z[f"adam/{n}/exp_avg"],
                                   rtol=1e-3, atol=1e-7, err_msg=n)
        assert float(st["step"]) == float(z[f"adam/{names[0]}/step"])
    if bool(z["cfg/decay_lr"]):
        assert abs(agent.optimizer.param_groups[0]["lr"] - float(z[f"lr_after{n_learn - 1}"])) < 1e-12


@pytest.mark.parametrize("name", ["cartpole_small", "lunar_medium", "cheetah_small"])
def test_minibatch_gradient_matches_reference(name):
    """First minibatch gradient (pre-clip) through dppo_minibatch_grad_f32."""
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, _ = (int(x) for x in z["dims"])
    agent = make_agent(z)
    L = agent._learner
    h = L.handle
    hp = diamond.engine.hparams(agent.cfg, agent.cfg.lr, 0)
    ro = diamond.engine.stage_experience(experience(z, 0), dev(), bool(cont))
    N.check(h.lib.dppo_prepare_f32(h.h, ctypes.byref(ro.as_struct()), L.flat.flat.data_ptr(),
                                   ctypes.byref(hp), None, stream()))
    B = T * Nn
    mb = B // agent.cfg.num_minibatches
    idx = t(z["perms"][0][:mb], torch.int32)
    g = torch.zeros(L.flat.total, device=dev())
    loss4 = (ctypes.c_float * 4)()
    N.check(h.lib.dppo_minibatch_grad_f32(h.h, L.flat.flat.data_ptr(), idx.data_ptr(), mb, mb,
                                          ctypes.byref(hp), g.data_ptr(), loss4, stream()))
    torch.cuda.synchronize()
    gl = g.cpu().numpy()
    Lay = h.layout
    got = np.concatenate([gl[Lay.offset[i]:Lay.offset[i] + Lay.numel[i]] for i in range(Lay.count)])
    ref = z["grads"][0]
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 2e-5 * scale, np.abs(got - ref).max() / scale
    assert abs(loss4[0] - z["loss"][0]) <= 2e-5 * max(1, abs(z["loss"][0]))


def test_gae_kernel_via_agent_api():
    """PPO.calculate_advantage accepts the reference's float 0/1 term/trunc tensors."""
    z = load_golden("learn_cartpole_small.npz")
    agent = make_agent(z)
    d = load_golden("gae_cases.npz")
    n = "random_16x8"
    T, Nn = d[n + "/rewards"].shape
    agent.cfg.rollout_steps = T
    adv = agent.calculate_advantage(torch.from_numpy(d[n + "/rewards"]),
                                    torch.from_numpy(d[n + "/term"].astype(np.float32)),
                                    torch.from_numpy(d[n + "/trunc"].astype(np.float32)),
                                    torch.from_numpy(d[n + "/values"]),
                                    torch.from_numpy(d[n + "/next_values"]))
    assert np.array_equal(adv.cpu().numpy(), d[n + "/adv"])


def test_learn_large_vs_oracle():
    """CartPole-shaped learn at N=256 (B=32,768) against the NumPy oracle, same perms."""
    from oracle import ppo_np as P
    import gym_stub
    T, Nn, D, A = 128, 256, 4, 2
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=Nn, verbose=False)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * Nn)
    agent = diamond.PPO(None, cfg, envs=envs)
    names = [n for n, _ in agent.network.named_parameters()]
    params = {n: p.detach().cpu().numpy().copy() for n, p in agent.network.named_parameters()}
    rng = np.random.default_rng(0)
    exp = [[rng.standard_normal((Nn, D)).astype(np.float32),
            rng.standard_normal((Nn, D)).astype(np.float32),
            rng.integers(0, A, Nn), rng.normal(1, 1, Nn), rng.random(Nn) < 0.02,
            rng.random(Nn) < 0.005] for _ in range(T)]
    st = np.random.get_state()
    agent.learn(exp)
    tr = agent.learn_trace()
    np.random.set_state(st)
    hp = P.Hyper()
    adam = P.new_adam_state(params, names)
    stacked = [np.asarray(x) for x in zip(*exp)]
    ref = P.learn(params, adam, stacked, hp, cfg.lr, False, rng=np.random)
    np.testing.assert_allclose(tr[:, 0], ref["loss"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(tr[:, 4], ref["norm"], rtol=1e-4, atol=1e-5)
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), params[n], rtol=0, atol=2e-5,
                                   err_msg=n)


def test_learn_is_deterministic():
    z = load_golden("learn_lunar_medium.npz")
    res = []
    for _ in range(2):
        agent = make_agent(z)
        np.random.set_state(("MT19937", z["rng_state_before0"].astype(np.uint32),
                             int(z["rng_pos_before0"]), 0, 0.0))
        ro = diamond.engine.stage_experience(experience(z, 0), dev(), False)
        agent.learn_device(ro)
        torch.cuda.synchronize()
        res.append(flat_params(agent))
    assert np.array_equal(res[0], res[1])


def test_agent_teardown_drains_permutation_drafts():
    """An agent dropped right after a learn() (its look-ahead drafts still queued or swapping on
    the host pool into the handle's pinned slots) is garbage-collected: the learner drains the
    drafts before dppo_destroy frees the slots, its draft thread ends, and the next agent works.
    Also explicit close() on a live agent, twice."""
    import gc
    import weakref
    z = load_golden("learn_lunar_medium.npz")
    results = []
    for k in range(3):
        agent = make_agent(z)
        np.random.seed(21)
        agent.learn(experience(z, 0))
        assert agent._learner._drafts            # drafts for the next learns are in flight
        results.append(flat_params(agent))
        worker = agent._learner._worker
        if k == 2:
            agent.close()
            agent.close()
            assert not worker._thread.is_alive()
            continue
        ref = weakref.ref(agent._learner)
        del agent
        gc.collect()
        assert ref() is None, "the learner was kept alive"
        worker._thread.join(30)
        assert not worker._thread.is_alive()
    assert np.array_equal(results[0], results[1]) and np.array_equal(results[0], results[2])


def test_indivisible_minibatch_raises_value_error():
    import gym_stub
    cfg = diamond.PPOConfig(rollout_steps=3, num_envs=5, num_minibatches=4, verbose=False)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(4, 2)] * 5)
    agent = diamond.PPO(None, cfg, envs=envs)
    rng = np.random.default_rng(0)
    exp = [[rng.standard_normal((5, 4)).astype(np.float32), rng.standard_normal((5, 4)).astype(np.float32),
            rng.integers(0, 2, 5), rng.normal(size=5), rng.random(5) < 0.1, rng.random(5) < 0.1]
           for _ in range(3)]
    with pytest.raises(ValueError):
        agent.learn(exp)


@pytest.mark.parametrize("walk", ["1", "0"])
@pytest.mark.parametrize("n,count", [(1, 1), (2, 3), (3, 4), (17, 2), (1000, 4), (65539, 2),
                                     (524288, 4)])
def test_device_fisher_yates_resolution_matches_numpy(monkeypatch, walk, n, count):
    """dppo_perm_resolve(host MT19937 targets) == np.random.permutation, bit-exact: by the value
    walk (DPPO_PERM_WALK=1, default) and by the links + chain passes (=0)."""
    monkeypatch.setenv("DPPO_PERM_WALK", walk)
    np.random.seed(1000 + n)
    key, pos, _ = N.mt_state()
    tg = np.empty(count * n, np.int32)
    N.perm_targets_numpy(key, pos, n, count, tg)
    np.random.seed(1000 + n)
    ref = np.concatenate([np.random.permutation(n) for _ in range(count)]).astype(np.int32)
    td = t(tg, torch.int32)
    out = torch.full((count * n,), -7, dtype=torch.int32, device=dev())
    scratch = torch.empty(3 * count * n, dtype=torch.int32, device=dev())
    N.perm_resolve(td.data_ptr(), out.data_ptr(), n, count, scratch.data_ptr(), stream())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


def _fisher_yates(j):
    a = np.arange(len(j), dtype=np.int32)
    for i in range(len(j) - 1, 0, -1):
        k = int(j[i])
        a[i], a[k] = a[k], a[i]
    return a


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("n,count", [(1000, 4), (65539, 2), (524288, 4)])
def test_device_resolution_packed_and_public_scratch_match_numpy(monkeypatch, packed, n, count):
    """dppo_perm_resolve_ex with the packed-pair scratch (dppo_perm_resolve_scratch: the handle's
    own form) and with the public 3 * count * n: both equal np.random.permutation, bit-exact."""
    monkeypatch.setenv("DPPO_PERM_WALK", "0")
    np.random.seed(2000 + n)
    key, pos, _ = N.mt_state()
    tg = np.empty(count * n, np.int32)
    N.perm_targets_numpy(key, pos, n, count, tg)
    np.random.seed(2000 + n)
    ref = np.concatenate([np.random.permutation(n) for _ in range(count)]).astype(np.int32)
    ints = N.perm_resolve_scratch(n, count) if packed else 3 * count * n
    assert ints >= 3 * count * n
    out = torch.full((count * n,), -7, dtype=torch.int32, device=dev())
    scratch = torch.empty(ints, dtype=torch.int32, device=dev())
    N.perm_resolve_ex(t(tg, torch.int32).data_ptr(), out.data_ptr(), n, count, scratch.data_ptr(),
                      ints, stream())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("kind", ["zeros", "identity", "shifted"])
def test_device_resolution_on_adversarial_targets(monkeypatch, packed, kind):
    """Valid but adversarial swap targets (every j_i <= i is a Fisher-Yates input): all zero -- one
    bucket of n - 1 steps, sorted in place in O(m log m) --, identity, shifted; the sequential
    loop's permutation, bit-exact, on both scratch forms and within the test's time limit."""
    monkeypatch.setenv("DPPO_PERM_WALK", "0")
    n, count = 65539, 2
    i = np.arange(n)
    j = {"zeros": np.zeros(n), "identity": i, "shifted": np.maximum(i - 1, 0)}[kind].astype(np.int32)
    tg = np.concatenate([j] * count)
    ref = np.concatenate([_fisher_yates(j)] * count)
    ints = N.perm_resolve_scratch(n, count) if packed else 3 * count * n
    out = torch.full((count * n,), -7, dtype=torch.int32, device=dev())
    scratch = torch.empty(ints, dtype=torch.int32, device=dev())
    N.perm_resolve_ex(t(tg, torch.int32).data_ptr(), out.data_ptr(), n, count, scratch.data_ptr(),
                      ints, stream())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("device_shuffle", [False, True])
def test_permutation_lookahead_hit_and_miss(device_shuffle):
    """The next learn's permutations are drawn ahead on a host thread; they are used only while
    the global NumPy RNG is untouched.  Interleaving foreign np.random draws must give exactly the
    results of a learner without look-ahead, and leave the same RNG state -- with the swaps on
    the host or resolved on the device."""
    z = load_golden("learn_lunar_medium.npz")
    results = []
    for lookahead in (True, False):
        agent = make_agent(z)
        agent._learner.lookahead = lookahead
        agent._learner.device_shuffle = device_shuffle
        np.random.seed(11)
        ro = diamond.engine.stage_experience(experience(z, 0), dev(), False)
        agent.learn_device(ro)            # draws its own; the draft for learn 2 starts
        agent.learn_device(ro)            # hit
        np.random.random(3)               # foreign draw: the draft for learn 3 is now stale
        agent.learn_device(ro)            # miss -> redrawn from the live state
        agent.learn_device(ro)            # hit
        torch.cuda.synchronize()
        st = np.random.get_state()
        results.append((flat_params(agent), st[1].copy(), st[2],
                        agent._learner.host_seconds["lookahead_hits"]))
    (p1, k1, q1, hits1), (p2, k2, q2, hits2) = results
    assert np.array_equal(p1, p2)
    assert np.array_equal(k1, k2) and q1 == q2
    assert hits1 == 2 and hits2 == 0


# ---------------------------------------------------------------------------------------------
def test_tanh_squash_rollout_and_learn():
    """ContinuousPPOConfig.tanh_squash (extension): the env receives tanh(u) rescaled
    to the Box bounds -- computed on the device by the act kernel -- and checked against the
    oracle's squash_action of the experience's Gaussian samples u; learn() on that experience is
    bit-identical to the unsquashed agent's learn() on the same experience (the squash's
    log-density correction does not depend on the parameters)."""
    from oracle import ppo_np as P
    import gym_stub

    class RecordingEnvs(gym_stub.SyncVectorEnv):
        def step(self, actions):
            self.sent.append(np.array(actions, copy=True))
            return super().step(actions)

    T, Nn, D, A = 8, 16, 5, 3
    params = []
    squashed_exp = None
    for squash in (True, False):
        np.random.seed(0)
        torch.manual_seed(0)
        envs = RecordingEnvs([lambda: gym_stub.SyntheticEnv(D, 1, continuous=True, act_dim=A)] * Nn)
        envs.single_action_space.low = -2.0
        envs.single_action_space.high = 2.0
        envs.sent = []
        cfg = diamond.ContinuousPPOConfig(rollout_steps=T, num_envs=Nn, verbose=False,
                                          tanh_squash=squash)
        agent = diamond.ContinuousPPO(None, cfg, envs=envs)
        agent.current_observations, _ = envs.reset(seed=3)
        exp = agent.rollout()
        u = np.stack([e[2] for e in exp])
        sent = np.stack(envs.sent)
        if squash:
            assert np.all(np.abs(sent) <= 2.0)
            np.testing.assert_allclose(sent, P.squash_action(u, -2.0, 2.0), rtol=0, atol=2e-6)
            assert not np.allclose(sent, u)
            squashed_exp = exp
        else:
            np.testing.assert_array_equal(sent, u)
        np.random.seed(7)
        agent.learn(squashed_exp)
        torch.cuda.synchronize()
        params.append(flat_params(agent))
    np.testing.assert_array_equal(params[0], params[1])


@pytest.mark.parametrize("continuous", [False, True])
def test_staged_rollout_learn_matches_unstaged(continuous):
    """rollout() stages every step into HBM as the envs step (RolloutStager);
    learn() of the returned list must equal learn() of the same experience stacked and uploaded
    the reference way -- also when the list handed to learn() is a different object (re-staged),
    and across consecutive rollouts (the two staging slots alternate)."""
    import gym_stub
    T, Nn, D, A = 16, 32, 6, 3
    results = []
    for mode in ("staged", "unstaged", "copy"):
        np.random.seed(0)
        torch.manual_seed(0)
        envs = gym_stub.SyncVectorEnv(
            [lambda: gym_stub.SyntheticEnv(D, A, continuous=continuous, act_dim=A)] * Nn)
        Cfg = diamond.ContinuousPPOConfig if continuous else diamond.PPOConfig
        Agent = diamond.ContinuousPPO if continuous else diamond.PPO
        agent = Agent(None, Cfg(rollout_steps=T, num_envs=Nn, verbose=False), envs=envs)
        agent.stage_rollout = mode != "unstaged"
        agent.current_observations, _ = envs.reset(seed=5)
        for _ in range(3):
            exp = agent.rollout()
            agent.learn(list(exp) if mode == "copy" else exp)
        torch.cuda.synchronize()
        results.append(flat_params(agent))
    np.testing.assert_array_equal(results[0], results[1])
    np.testing.assert_array_equal(results[2], results[1])


# ---------------------------------------------------------------------------------------------
def _act_agent(continuous, D, A, Nn):
    import gym_stub
    np.random.seed(0)
    torch.manual_seed(0)
    envs = gym_stub.SyncVectorEnv(
        [lambda: gym_stub.SyntheticEnv(D, A, continuous=continuous, act_dim=A)] * Nn)
    Cfg = diamond.ContinuousPPOConfig if continuous else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if continuous else diamond.PPO
    return Agent(None, Cfg(rollout_steps=8, num_envs=Nn, verbose=False), envs=envs)


def test_act_and_squash_samplers_share_one_call_counter():
    """act() and the squashing sampler draw from ONE Philox call counter: with the same seed, a
    squashed call followed by an unsquashed one uses distinct draws (rewinding the counter
    reproduces the squashed call's u)."""
    D, A, n = 17, 6, 4096
    agent = _act_agent(True, D, A, 64)
    obs = np.random.default_rng(5).standard_normal((n, D)).astype(np.float32)
    u1, _ = agent._learner.act(obs, 99, squash=True)
    u2 = agent._learner.act(obs, 99)
    assert not np.array_equal(u1, u2)
    agent._learner._act_counter -= 2
    u3, _ = agent._learner.act(obs, 99, squash=True)
    assert np.array_equal(u1, u3)


def test_fused_actions_categorical_distribution():
    """dppo_act_f32 (rollout sampling, replaces get_actions ppo.py:73-82): deterministic per
    (seed, counter), and its empirical action frequencies for one observation repeated 2^17 times
    match the network's softmax probabilities within 5 sigma."""
    D, A, n = 8, 4, 1 << 17
    agent = _act_agent(False, D, A, 64)
    with torch.no_grad():
        agent.network.actor_out_layer.weight.mul_(100.0)   # spread the probabilities out
    rng = np.random.default_rng(3)
    o = rng.standard_normal(D).astype(np.float32)
    obs = np.tile(o, (n, 1))
    a1 = agent._learner.act(obs, 1234)
    agent._learner._act_counter -= 1
    a2 = agent._learner.act(obs, 1234)
    a3 = agent._learner.act(obs, 1234)
    assert a1.dtype == np.int64 and np.array_equal(a1, a2) and not np.array_equal(a2, a3)
    with torch.no_grad():
        logits, _ = agent.network.get_logits_and_values(torch.from_numpy(o).to(dev())[None])
        p = torch.softmax(logits[0].double(), -1).cpu().numpy()
    assert p.min() > 0.01 and p.max() < 0.97
    freq = np.bincount(a1, minlength=A) / n
    sig = np.sqrt(p * (1 - p) / n)
    assert np.all(np.abs(freq - p) <= 5 * sig + 1e-12), (freq, p)
    assert a1.min() >= 0 and a1.max() < A


def test_fused_actions_gaussian_mean_and_scale():
    """Continuous sampling: with log_std = -30 the samples ARE the actor means (checks the fused
    forward against the torch module); with log_std = -0.5 the per-dimension sample mean and std
    of 2^17 draws for one observation match mean / exp(log_std) within 5 sigma."""
    D, A, n = 17, 6, 1 << 17
    agent = _act_agent(True, D, A, 64)
    rng = np.random.default_rng(4)
    obs = rng.standard_normal((4096, D)).astype(np.float32)
    with torch.no_grad():
        agent.network.actor_log_std.fill_(-30.0)
        mean, _, _ = agent.network.get_means_log_stds_and_values(torch.from_numpy(obs).to(dev()))
    acts = agent._learner.act(obs, 99)
    assert acts.dtype == np.float32 and acts.shape == (4096, A)
    np.testing.assert_allclose(acts, mean.cpu().numpy(), rtol=0, atol=2e-5)
    with torch.no_grad():
        agent.network.actor_log_std.fill_(-0.5)
    o = obs[:1]
    with torch.no_grad():
        mu = agent.network.get_means_log_stds_and_values(torch.from_numpy(o).to(dev()))[0][0]
    mu = mu.cpu().numpy().astype(np.float64)
    x = agent._learner.act(np.tile(o, (n, 1)), 7).astype(np.float64)
    sd = np.exp(-0.5)
    assert np.all(np.abs(x.mean(0) - mu) <= 5 * sd / np.sqrt(n))
    assert np.all(np.abs(x.std(0) - sd) <= 5 * sd / np.sqrt(2 * n))


# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["cartpole_small", "cheetah_small"])
def test_generic_network_path_matches_reference_trace(name):
    """A custom network_cls (here a subclass of the default network, which the fused kernels do
    not claim) takes the generic path: the module under torch autograd on the GPU, GAE /
    normalisation / clip + Adam in the HIP kernels.  It must reproduce the reference's captured
    learn() like the fused path does."""
    z = load_golden(f"learn_{name}.npz")
    T, Nn, D, A, cont, n_learn = (int(x) for x in z["dims"])
    base = diamond.continuous_ppo.ContinuousActorCriticNetwork if cont else \
        diamond.ppo.ActorCriticNetwork

    class CustomNet(base):
        pass

    import gym_stub
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    kw = {k: z["cfg/" + k].item() for k in ("num_epochs", "num_minibatches", "lr", "adam_eps",
                                             "gamma", "gae_lambda", "ppo_clip",
                                             "value_loss_weight", "entropy_beta",
                                             "grad_norm_clip", "total_steps")}
    cfg = Cfg(rollout_steps=T, num_envs=Nn, verbose=False,
              advantage_norm=bool(z["cfg/advantage_norm"]), decay_lr=bool(z["cfg/decay_lr"]), **kw)
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A, continuous=bool(cont),
                                                                 act_dim=A)] * Nn)
    agent = Agent(None, cfg, network_cls=CustomNet, envs=envs)
    assert not agent._learner.fused
    sd = {n: torch.from_numpy(z["init/" + n]) for n in z["param_names"]}
    if hasattr(agent.network, "actor_out_layer"):
        sd["actor_out_layer.weight"] = sd["actor_head.2.weight"]
        sd["actor_out_layer.bias"] = sd["actor_head.2.bias"]
    agent.network.load_state_dict(sd)
    for li in range(n_learn):
        np.random.set_state(("MT19937", z[f"rng_state_before{li}"].astype(np.uint32),
                             int(z[f"rng_pos_before{li}"]), 0, 0.0))
        agent.learn(experience(z, li))
        torch.cuda.synchronize()
    for n, p in agent.network.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0, atol=5e-6,
                                   err_msg=n)


def test_checkpoint_roundtrip_continues_identically():
    """Checkpointer (utils.py:584-619 format) save -> load_checkpoint into a fresh agent -> the
    next learn() gives bit-identical parameters and Adam moments to the uninterrupted agent."""
    import tempfile
    z = load_golden("learn_lunar_medium.npz")
    a1 = make_agent(z)
    np.random.seed(3)
    a1.learn(experience(z, 0))
    torch.cuda.synchronize()
    with tempfile.TemporaryDirectory() as d:
        a1.checkpointer.folder = __import__("pathlib").Path(d)
        a1.checkpointer.save(1, a1.network, a1.optimizer)
        path = sorted(__import__("pathlib").Path(d).glob("*.pt"))[0]
        a2 = make_agent(z)
        a2.load_checkpoint(path)
    st = np.random.get_state()
    a1.learn(experience(z, 0))
    np.random.set_state(st)
    a2.learn(experience(z, 0))
    torch.cuda.synchronize()
    assert np.array_equal(flat_params(a1), flat_params(a2))
    for p1, p2 in zip(a1.network.parameters(), a2.network.parameters()):
        s1, s2 = a1.optimizer.state[p1], a2.optimizer.state[p2]
        assert torch.equal(s1["exp_avg"], s2["exp_avg"])
        assert torch.equal(s1["exp_avg_sq"], s2["exp_avg_sq"])
        assert float(s1["step"]) == float(s2["step"])


def test_recurrent_ppo_rollout_and_learn_run():
    """RecurrentPPO (the reference's crashes at recurrent_ppo.py:78; intended semantics here):
    train() -- rollout() and learn() -- runs on the stub env, changes the parameters, keeps them
    finite, and its calculate_advantage is the bit-exact GAE kernel."""
    import gym_stub
    from oracle import ppo_np as P
    np.random.seed(0)
    torch.manual_seed(0)
    T, Nn, D, A = 16, 8, 4, 2
    envs = gym_stub.SyncVectorEnv([lambda: gym_stub.SyntheticEnv(D, A)] * Nn)
    cfg = diamond.RecurrentPPOConfig(rollout_steps=T, num_envs=Nn, verbose=False, num_epochs=2,
                                     total_steps=2 * T * Nn)
    agent = diamond.RecurrentPPO(None, cfg, envs=envs)
    before = flat_params(agent)
    agent.train()  # two rollout() + learn() iterations
    torch.cuda.synchronize()
    after = flat_params(agent)
    assert np.all(np.isfinite(after)) and not np.array_equal(before, after)
    rng = np.random.default_rng(2)
    r = rng.normal(1, 1, (T, Nn)).astype(np.float32)
    te = (rng.random((T, Nn)) < 0.1).astype(np.float32)
    tr = (rng.random((T, Nn)) < 0.05).astype(np.float32)
    v = rng.standard_normal((T, Nn)).astype(np.float32)
    nv = rng.standard_normal((T, Nn)).astype(np.float32)
    adv = agent.calculate_advantage(torch.from_numpy(r), torch.from_numpy(te),
                                    torch.from_numpy(tr), torch.from_numpy(v),
                                    torch.from_numpy(nv))
    assert np.array_equal(adv.cpu().numpy(), P.gae(r, te, tr, v, nv))


@pytest.mark.parametrize("cont", [False, True])
def test_loopback_two_ranks_match_union_minibatch_learn(cont):
    """The data-parallel learn with world_size 2 on ONE device: two handles in a
    loopback group (dppo_loopback_group: every exchange RCCL would carry -- advantage (sum, sum^2),
    per-minibatch gradient + loss partials -- summed on the device) driven concurrently from two
    threads, each rank owning half the envs and its own permutations.  Oracle: ONE learn of the
    global batch whose minibatch j is the union of the ranks' local minibatches j (global
    advantage statistics, global divisors, continuous entropy constant once)."""
    import threading
    from oracle import ppo_np as P
    T, Nl, world, E, M = 16, 32, 2, 4, 8
    D, A = (17, 6) if cont else (4, 2)
    Ng, B = Nl * world, T * Nl
    mb = B // M
    rng = np.random.default_rng(5)
    obs = rng.standard_normal((T, Ng, D)).astype(np.float32)
    nobs = rng.standard_normal((T, Ng, D)).astype(np.float32)
    act = (rng.standard_normal((T, Ng, A)).astype(np.float32) if cont
           else rng.integers(0, A, (T, Ng)))
    rew = rng.normal(1, 1, (T, Ng)).astype(np.float32)
    te, tr = rng.random((T, Ng)) < 0.05, rng.random((T, Ng)) < 0.02
    handles = [N.Handle(0, N.Dims(T, Nl, D, A, int(cont), 64, E, M, world, r))
               for r in range(world)]
    L = handles[0].layout
    names = P.CONTINUOUS_NAMES if cont else P.DISCRETE_NAMES
    params = {}
    for i, n in enumerate(names):
        shp = (L.rows[i],) if n.endswith("bias") else (L.rows[i], L.cols[i])
        params[n] = (rng.standard_normal(shp) * 0.3).astype(np.float32)
    flat0 = np.zeros(L.total, np.float32)
    for i, n in enumerate(names):
        flat0[L.offset[i]:L.offset[i] + L.numel[i]] = params[n].ravel()
    N.loopback_group(handles)
    perms = [np.stack([np.random.RandomState(100 + r).permutation(B) for _ in range(E)])
             .astype(np.int32) for r in range(world)]
    hp = N.HParams(gamma=0.99, gae_lambda=0.95, ppo_clip=0.2, value_loss_weight=1.0,
                   entropy_beta=0.01, grad_norm_clip=0.5, adam_beta1=0.9, adam_beta2=0.999,
                   adam_eps=1e-5, advantage_norm=1, lr=3e-4, adam_step=0)
    state = []
    for r in range(world):
        sl = slice(r * Nl, (r + 1) * Nl)
        exp = [[obs[k, sl], nobs[k, sl], act[k, sl], rew[k, sl], te[k, sl], tr[k, sl]]
               for k in range(T)]
        ro = diamond.engine.stage_experience(exp, dev(), cont)
        state.append({"ro": ro, "st": ro.as_struct(), "p": t(flat0),
                      "m": torch.zeros(L.total, device=dev()),
                      "v": torch.zeros(L.total, device=dev()), "rc": None})
    torch.cuda.synchronize()

    def run(r):
        torch.cuda.set_device(0)
        s = torch.cuda.Stream(device=dev())
        x = state[r]
        x["rc"] = handles[r].lib.dppo_learn_f32(
            handles[r].h, ctypes.byref(x["st"]), x["p"].data_ptr(), x["m"].data_ptr(),
            x["v"].data_ptr(), ctypes.byref(hp), perms[r].ctypes.data, None, s.cuda_stream)
        s.synchronize()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=150)
    assert all(not x.is_alive() for x in th)
    for x in state:
        N.check(x["rc"], "dppo_learn_f32 (loopback rank)")
    torch.cuda.synchronize()
    # the oracle: global batch, minibatch j = union of the ranks' local minibatches j
    to_global = lambda r, i: (i // Nl) * Ng + r * Nl + i % Nl
    perms_g = np.stack([np.concatenate([to_global(r, perms[r][e, j * mb:(j + 1) * mb])
                                        for j in range(M) for r in range(world)])
                        for e in range(E)])
    adam = P.new_adam_state(params, names)
    ref = P.learn(params, adam, [obs, nobs, act, rew, te, tr], P.Hyper(), 3e-4, cont,
                  perms=perms_g)
    flats = [x["p"].cpu().numpy() for x in state]
    assert np.array_equal(flats[0], flats[1])  # replicated clip + Adam on identical sums
    # Tolerances: the N(0, 0.3^2) random init gives pre-clip gradient norms of 20-50 (clipped to
    # 0.5 every step); the two-rank sum re-associates each minibatch's gradient, and over 32 Adam
    # steps that drift reaches ~5e-4 relative in the continuous grad norms (the one-device split
    # path matches the reference traces at 2e-5, test_learn_matches_reference_trace).
    for r in range(world):
        tr_r = handles[r].trace(E * M)
        np.testing.assert_allclose(tr_r[:, 0], ref["loss"], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(tr_r[:, 4], ref["norm"], rtol=2e-3, atol=1e-5)
    for i, n in enumerate(names):
        np.testing.assert_allclose(flats[0][L.offset[i]:L.offset[i] + L.numel[i]],
                                   params[n].ravel(), rtol=0, atol=5e-5, err_msg=n)
