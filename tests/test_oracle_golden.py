"""Pin the CPU oracle against golden fixtures captured from the reference (CPU-only tests).

Tolerances: GAE is bit-exact (same fp32 op order, reference ppo.py:201-220); everything
downstream of a reduction is tolerance-based (SURVEY.md §7.2 hard part 2).
"""
import numpy as np
import pytest

from conftest import LEARN_TRACES, load_golden
from oracle import ppo_np as P
from oracle.mt19937 import MT19937


def test_gae_bitexact_all_cases():
    d = load_golden("gae_cases.npz")
    for n in d["names"]:
        adv = P.gae(d[n + "/rewards"], d[n + "/term"], d[n + "/trunc"], d[n + "/values"],
                    d[n + "/next_values"])
        assert np.array_equal(adv, d[n + "/adv"]), n
        ret = d[n + "/values"] + adv
        assert np.array_equal(ret, d[n + "/returns"]), n


def test_adv_normalisation():
    d = load_golden("gae_cases.npz")
    for n in d["names"]:
        adv = d[n + "/adv"]
        if adv.size < 2:
            continue
        mean, std = P.adv_stats(adv)
        assert abs(mean - d[n + "/mean"]) <= 1e-6 * max(1, abs(d[n + "/mean"])), n
        assert abs(std - d[n + "/std"]) <= 1e-6 * d[n + "/std"], n
        np.testing.assert_allclose(P.normalize_adv(adv), d[n + "/adv_norm"], rtol=0, atol=1e-6)


def test_gae_properties():
    rng = np.random.default_rng(0)
    T, N = 33, 5
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    nv = rng.normal(size=(T, N)).astype(np.float32)
    z = np.zeros((T, N), np.uint8)
    # no dones: adv_t = sum_k (g l)^k delta_{t+k}
    adv = P.gae(r, z, z, v, nv)
    g, c = 0.99, 0.99 * 0.95
    delta = r.astype(np.float64) + g * nv - v
    ref = np.zeros_like(delta)
    a = 0.0
    for t in range(T - 1, -1, -1):
        a = delta[t] + c * a
        ref[t] = a
    np.testing.assert_allclose(adv, ref, rtol=1e-5, atol=1e-5)
    # all terminated: adv = r - v
    o = np.ones((T, N), np.uint8)
    np.testing.assert_array_equal(P.gae(r, o, z, v, nv), r - v)
    # all truncated: adv = r + g*nv - v (bootstrap kept, lambda-chain cut)
    np.testing.assert_array_equal(P.gae(r, z, o, v, nv),
                                  (r + np.float32(g) * nv) - v)


def test_permutation_restatement_matches_numpy_and_golden():
    d = load_golden("perm_seed42.npz")
    np.random.seed(42)
    g = MT19937.from_numpy_state(np.random.get_state())
    assert np.array_equal(g.permutation(1024), d["p1024"])
    assert list(d["p1024"][:8]) == [525, 357, 444, 31, 618, 587, 447, 734]
    assert np.array_equal(g.permutation(7), d["p7"])
    assert np.array_equal(g.permutation(1), d["p1"])


def _hyper(z):
    keys = ["gamma", "gae_lambda", "num_epochs", "num_minibatches", "ppo_clip",
            "value_loss_weight", "entropy_beta", "grad_norm_clip", "lr", "adam_eps"]
    return P.Hyper(**{k: z["cfg/" + k].item() for k in keys},
                   advantage_norm=bool(z["cfg/advantage_norm"]))


def replay_trace(z):
    """Run the oracle through every learn() of a golden trace with the captured perms."""
    T, N, D, A, cont, n_learn = (int(x) for x in z["dims"])
    names = list(z["param_names"])
    params = {n: z["init/" + n].copy() for n in names}
    hp = _hyper(z)
    adam = P.new_adam_state(params, names)
    lr, E = hp.lr, hp.num_epochs
    out = {"loss": [], "norm": [], "grads": [], "params": [], "old": []}
    for li in range(n_learn):
        exp = [z[f"exp{li}/" + k] for k in ("obs", "next_obs", "actions", "rewards", "term", "trunc")]
        tr = P.learn(params, adam, exp, hp, lr, bool(cont), perms=z["perms"][li * E:(li + 1) * E],
                     record=True)
        for k in ("loss", "norm", "grads", "params"):
            out[k] += tr[k]
        out["old"].append(tr)
        if bool(z["cfg/decay_lr"]):
            lr = P.linear_lr_factor_step(lr, li + 1, int(z["cfg/total_steps"]) // (T * N), 1.0, 0.05)
    return params, adam, out, names


@pytest.mark.parametrize("name", LEARN_TRACES)
def test_learn_trace(name):
    z = load_golden(f"learn_{name}.npz")
    params, adam, out, names = replay_trace(z)
    for li, tr in enumerate(out["old"]):
        np.testing.assert_allclose(tr["old_logp"], z["old/log_probs"][li], atol=1e-5)
        np.testing.assert_allclose(tr["values"], z["old/values"][li], atol=1e-5)
        np.testing.assert_allclose(tr["next_values"], z["old/next_values"][li], atol=1e-5)
    np.testing.assert_allclose(out["loss"], z["loss"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["norm"], z["norm"], rtol=1e-5, atol=1e-5)
    ks = z["kept_steps"]
    g = np.stack(out["grads"])[ks]
    scale = np.abs(z["grads"]).max(axis=1, keepdims=True)
    assert (np.abs(g - z["grads"]) / scale).max() < 1e-5
    np.testing.assert_allclose(np.stack(out["params"])[ks], z["params"], rtol=0, atol=2e-6)
    for n in names:
        np.testing.assert_allclose(params[n], z["final/" + n], rtol=0, atol=2e-6)
        np.testing.assert_allclose(adam["m"][n], z[f"adam/{n}/exp_avg"], rtol=1e-4, atol=1e-8)
        np.testing.assert_allclose(adam["v"][n], z[f"adam/{n}/exp_avg_sq"], rtol=1e-4, atol=1e-10)
    assert adam["step"] == float(z[f"adam/{names[0]}/step"])


@pytest.mark.parametrize("name", ["cartpole_small", "lunar_medium", "cheetah_small",
                                  "pendulum_medium", "lunar_noadvnorm"])
def test_torch_cpu_restatement_matches_trace(name):
    """oracle/ppo_torch.py (bench.py's torch-CPU baseline) reproduces the reference's captured
    learn() traces: same losses, norms and final parameters."""
    from oracle import ppo_torch as PT
    z = load_golden(f"learn_{name}.npz")
    T, N, D, A, cont, n_learn = (int(x) for x in z["dims"])
    names = list(z["param_names"])
    params = {n: z["init/" + n].copy() for n in names}
    hp = _hyper(z)
    E = hp.num_epochs
    losses, norms, st = [], [], None
    for li in range(n_learn):
        exp = [z[f"exp{li}/" + k] for k in ("obs", "next_obs", "actions", "rewards", "term", "trunc")]
        tr = PT.learn(params, exp, hp, hp.lr, bool(cont), perms=z["perms"][li * E:(li + 1) * E],
                      adam_state=st)
        st = tr["adam_state"]
        losses += tr["loss"]
        norms += tr["norm"]
    np.testing.assert_allclose(losses, z["loss"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(norms, z["norm"], rtol=1e-5, atol=1e-5)
    for n in names:
        np.testing.assert_allclose(params[n], z["final/" + n], rtol=0, atol=2e-6, err_msg=n)
