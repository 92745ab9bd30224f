"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Test infrastructure only.  Runs only where /root/reference exists (the survey container);
the fixtures it writes are small .npz files that travel with the repo, the reference does not.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is captured (SURVEY.md §8(c) "Golden vectors to generate & commit"):

* gae_cases.npz      -- PPO.calculate_advantage (reference diamond/ppo.py:188-222) on edge cases:
                        term&trunc same step, last-step done, all-done column, T=1, no dones,
                        and random T=128 x N=64; plus returns and normalised advantages
                        (ppo.py:241-243).
* learn_<name>.npz   -- full PPO.learn / ContinuousPPO.learn traces (ppo.py:224-287,
                        continuous_ppo.py:236-299): initial state_dict, experience, old-policy
                        outputs, advantages, the E x M permutation, per-minibatch loss, pre-clip
                        gradients, total grad norm, parameters after every optimizer step, final
                        Adam state.  Some traces call learn() twice (Adam step / RNG continuation,
                        decay_lr).
* learn_cartpole_c1.npz -- BASELINE configs[0] (CartPole, T=128, N=8) at full size.
* perm_seed42.npz    -- numpy legacy RandomState permutations (ppo.py:120-122,254).
* ckpt_cartpole-step000128.pt + ckpt_cartpole_resume.npz -- a checkpoint written by the
                        reference's Checkpointer.save after one learn(), and the learn() of a fresh
                        reference agent resumed from it (utils.py:584-612).

Capture is done by wrapping bound methods / module attributes at call time; no reference
file is modified.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, HERE)
    import gym_stub  # noqa: E402

    gym_stub.install()
    sys.path.insert(0, REF)
    import diamond  # noqa: E402
    import diamond.ppo as ref_ppo  # noqa: E402
    import diamond.continuous_ppo as ref_cppo  # noqa: E402

    return gym_stub, diamond, ref_ppo, ref_cppo


def synth_experience(rng, T, N, D, A, continuous, p_term, p_trunc):
    """SURVEY §8(d) synthetic inputs, shaped exactly like rollout() output (ppo.py:165-172)."""
    exp = []
    for _ in range(T):
        obs = rng.standard_normal((N, D)).astype(np.float32)
        nobs = rng.standard_normal((N, D)).astype(np.float32)
        if continuous:
            act = rng.standard_normal((N, A)).astype(np.float32)
        else:
            act = rng.integers(0, A, N).astype(np.int64)
        rew = rng.normal(1.0, 1.0, N)  # float64 like gymnasium
        term = rng.random(N) < p_term
        trunc = rng.random(N) < p_trunc
        exp.append([obs, nobs, act, rew, term, trunc])
    return exp


# ----------------------------------------------------------------------------------------------
def make_gae_cases(diamond, gym_stub):
    out = {}
    rng = np.random.default_rng(7)

    def run(name, rewards, term, trunc, values, next_values):
        T, N = rewards.shape
        cfg = diamond.PPOConfig(rollout_steps=T, num_envs=N, verbose=False)
        agent = diamond.PPO(lambda: gym_stub.SyntheticEnv(4, 2), cfg=cfg)
        tt = lambda x: torch.as_tensor(x, dtype=torch.float32)
        adv = agent.calculate_advantage(tt(rewards), tt(term), tt(trunc), tt(values),
                                        tt(next_values))
        vals = tt(values)
        ret = vals + adv
        norm = (adv - adv.mean()) / (adv.std() + 1e-6) if adv.numel() > 1 else adv
        out[f"{name}/rewards"] = rewards.astype(np.float32)
        out[f"{name}/term"] = term.astype(np.uint8)
        out[f"{name}/trunc"] = trunc.astype(np.uint8)
        out[f"{name}/values"] = values.astype(np.float32)
        out[f"{name}/next_values"] = next_values.astype(np.float32)
        out[f"{name}/adv"] = adv.numpy()
        out[f"{name}/returns"] = ret.numpy()
        out[f"{name}/adv_norm"] = norm.numpy()
        out[f"{name}/mean"] = np.float32(adv.mean().item())
        out[f"{name}/std"] = np.float32(adv.std().item()) if adv.numel() > 1 else np.float32(0)

    def rnd(T, N, pt, ptr):
        r = rng.normal(1, 1, (T, N)).astype(np.float32)
        te = rng.random((T, N)) < pt
        tr = rng.random((T, N)) < ptr
        v = rng.standard_normal((T, N)).astype(np.float32)
        nv = rng.standard_normal((T, N)).astype(np.float32)
        return r, te, tr, v, nv

    names = []
    r, te, tr, v, nv = rnd(16, 8, 0.2, 0.1)
    run("random_16x8", r, te, tr, v, nv); names.append("random_16x8")
    r, te, tr, v, nv = rnd(12, 8, 0.0, 0.0)
    te[5, :] = True; tr[5, :] = True          # term and trunc on the same step
    run("term_and_trunc_same_step", r, te, tr, v, nv); names.append("term_and_trunc_same_step")
    r, te, tr, v, nv = rnd(10, 8, 0.0, 0.0)
    te[-1, :4] = True; tr[-1, 4:] = True      # done on the last step
    run("last_step_done", r, te, tr, v, nv); names.append("last_step_done")
    r, te, tr, v, nv = rnd(10, 8, 0.1, 0.1)
    te[:, 2] = True; tr[:, 5] = True           # all-done columns
    run("all_done_columns", r, te, tr, v, nv); names.append("all_done_columns")
    r, te, tr, v, nv = rnd(1, 16, 0.3, 0.3)
    run("T1", r, te, tr, v, nv); names.append("T1")
    r, te, tr, v, nv = rnd(32, 8, 0.0, 0.0)
    run("no_dones", r, te, tr, v, nv); names.append("no_dones")
    r, te, tr, v, nv = rnd(128, 64, 0.02, 0.005)
    run("random_128x64", r, te, tr, v, nv); names.append("random_128x64")
    r, te, tr, v, nv = rnd(37, 67, 0.05, 0.05)   # ragged: N not a multiple of 64
    run("ragged_37x67", r, te, tr, v, nv); names.append("ragged_37x67")
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "gae_cases.npz"), **out)
    print("gae_cases.npz:", len(names), "cases")


# ----------------------------------------------------------------------------------------------
def make_learn_trace(diamond, gym_stub, name, *, continuous, T, N, D, A, n_learn=1,
                     cfg_over=None, p_term=0.1, p_trunc=0.05, save_all_grads=False):
    cfg_over = dict(cfg_over or {})
    Cfg = diamond.ContinuousPPOConfig if continuous else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if continuous else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=N, verbose=False, **cfg_over)
    agent = Agent(lambda: gym_stub.SyntheticEnv(D, A, continuous=continuous, act_dim=A), cfg=cfg)
    net, opt = agent.network, agent.optimizer
    names = [n for n, _ in net.named_parameters()]
    out = {"param_names": np.array(names)}
    for n, p in net.named_parameters():
        out[f"init/{n}"] = p.detach().numpy().copy()
    out["cfg"] = np.array(repr(cfg))
    for k in ("rollout_steps", "num_envs", "num_epochs", "num_minibatches", "lr", "adam_eps",
              "gamma", "gae_lambda", "ppo_clip", "value_loss_weight", "entropy_beta",
              "grad_norm_clip", "total_steps"):
        out[f"cfg/{k}"] = np.array(getattr(cfg, k))
    out["cfg/advantage_norm"] = np.array(cfg.advantage_norm)
    out["cfg/decay_lr"] = np.array(cfg.decay_lr)
    out["dims"] = np.array([T, N, D, A, int(continuous), n_learn])

    rec = {"loss": [], "norm": [], "grads": [], "params": [], "perm": [], "lr": []}
    state = {"in_learn": False}

    # -- wrappers ------------------------------------------------------------------------------
    real_perm = np.random.permutation

    def perm_wrap(n):
        p = real_perm(n)
        if state["in_learn"]:
            rec["perm"].append(p.copy())
        return p

    real_clip = torch.nn.utils.clip_grad_norm_

    def clip_wrap(params, max_norm, *a, **k):
        params = list(params)
        rec["grads"].append(np.concatenate([p.grad.detach().numpy().ravel().copy() for p in params]))
        tn = real_clip(params, max_norm, *a, **k)
        rec["norm"].append(float(tn))
        return tn

    real_backward = torch.Tensor.backward

    def backward_wrap(self, *a, **k):
        rec["loss"].append(float(self.detach()))
        return real_backward(self, *a, **k)

    real_step = opt.step

    def step_wrap(*a, **k):
        r = real_step(*a, **k)
        rec["params"].append(np.concatenate([p.detach().numpy().ravel().copy()
                                             for p in net.parameters()]))
        rec["lr"].append(opt.param_groups[0]["lr"])
        return r

    opt.step = step_wrap
    old = {}
    real_adv = agent.calculate_advantage

    def adv_wrap(rewards, terms, truncs, values, next_values):
        a = real_adv(rewards, terms, truncs, values, next_values)
        old.setdefault("values", []).append(values.numpy().copy())
        old.setdefault("next_values", []).append(next_values.numpy().copy())
        old.setdefault("adv", []).append(a.numpy().copy())
        return a

    agent.calculate_advantage = adv_wrap

    if continuous:
        real_mlv = net.get_means_log_stds_and_values

        def eval_wrap(x):
            r = real_mlv(x)
            if x.dim() == 3:  # old-policy evaluation over the full [T,N,D] buffer
                m, ls, v = r
                lp = diamond.continuous_ppo.JointNormal(loc=m, scale=ls.exp()).log_prob(
                    state["actions"])
                old.setdefault("log_probs", []).append(lp.detach().numpy().copy())
                old.setdefault("means", []).append(m.detach().numpy().copy())
            return r

        net.get_means_log_stds_and_values = eval_wrap
    else:
        real_lv = net.get_logits_and_values

        def eval_wrap(x):
            r = real_lv(x)
            if x.dim() == 3:
                lg, v = r
                lp = torch.distributions.Categorical(logits=lg).log_prob(state["actions"])
                old.setdefault("log_probs", []).append(lp.detach().numpy().copy())
                old.setdefault("logits", []).append(lg.detach().numpy().copy())
            return r

        net.get_logits_and_values = eval_wrap

    rng = np.random.default_rng(100 + T * 7 + N)
    np.random.permutation = perm_wrap
    torch.nn.utils.clip_grad_norm_ = clip_wrap
    torch.Tensor.backward = backward_wrap
    try:
        for li in range(n_learn):
            exp = synth_experience(rng, T, N, D, A, continuous, p_term, p_trunc)
            o, no, ac, rw, te, tr = zip(*exp)
            out[f"exp{li}/obs"] = np.asarray(o)
            out[f"exp{li}/next_obs"] = np.asarray(no)
            out[f"exp{li}/actions"] = np.asarray(ac)
            out[f"exp{li}/rewards"] = np.asarray(rw)
            out[f"exp{li}/term"] = np.asarray(te)
            out[f"exp{li}/trunc"] = np.asarray(tr)
            state["actions"] = torch.as_tensor(
                np.asarray(ac), dtype=torch.float32 if continuous else torch.int64)
            out[f"rng_state_before{li}"] = np.array(np.random.get_state()[1])
            out[f"rng_pos_before{li}"] = np.array(np.random.get_state()[2])
            state["in_learn"] = True
            agent.learn(exp)
            state["in_learn"] = False
            out[f"lr_after{li}"] = np.array(opt.param_groups[0]["lr"])
    finally:
        np.random.permutation = real_perm
        torch.nn.utils.clip_grad_norm_ = real_clip
        torch.Tensor.backward = real_backward

    for k, v in old.items():
        out[f"old/{k}"] = np.stack(v)
    out["perms"] = np.stack(rec["perm"]).astype(np.int64)
    out["loss"] = np.array(rec["loss"], dtype=np.float64)
    out["norm"] = np.array(rec["norm"], dtype=np.float64)
    out["lr_per_step"] = np.array(rec["lr"], dtype=np.float64)
    grads = np.stack(rec["grads"])
    params = np.stack(rec["params"])
    if save_all_grads:
        out["grads"] = grads
        out["params"] = params
    else:  # keep fixtures small: first three steps and the last step of every learn()
        per = len(grads) // n_learn
        keep = sorted(set([0, 1, 2] + [per * (i + 1) - 1 for i in range(n_learn)]))
        out["grads"] = grads[keep]
        out["params"] = params[keep]
        out["kept_steps"] = np.array(keep)
    for n, p in net.named_parameters():
        out[f"final/{n}"] = p.detach().numpy().copy()
    for i, p in enumerate(net.parameters()):
        st = opt.state[p]
        out[f"adam/{names[i]}/exp_avg"] = st["exp_avg"].numpy().copy()
        out[f"adam/{names[i]}/exp_avg_sq"] = st["exp_avg_sq"].numpy().copy()
        out[f"adam/{names[i]}/step"] = np.array(float(st["step"]))
    path = os.path.join(HERE, f"learn_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"learn_{name}.npz: {len(rec['loss'])} steps, {grads.shape[1]} params,"
          f" {os.path.getsize(path) // 1024} KiB")


def make_perm_golden():
    np.random.seed(42)
    p1024 = np.random.permutation(1024)
    p7 = np.random.permutation(7)
    p1 = np.random.permutation(1)
    big = np.random.permutation(1 << 17)
    st = np.random.get_state()
    np.savez_compressed(os.path.join(HERE, "perm_seed42.npz"), p1024=p1024, p7=p7, p1=p1,
                        big_head=big[:4096], big_sum_sq=np.array(int((big.astype(np.int64) ** 2
                                                                      * np.arange(big.size)).sum() % (1 << 61))),
                        state_after_keys=st[1], state_after_pos=np.array(st[2]))
    print("perm_seed42.npz; first 8 of permutation(1024):", p1024[:8])


def make_checkpoint_fixture(diamond, gym_stub):
    """A checkpoint written by the reference's own Checkpointer.save (utils.py:584-600) after one
    learn(), and the trace of a FRESH reference agent that Checkpointer.load-s it (utils.py:602-612)
    and learns on a second rollout: the oracle for resuming from a reference checkpoint.  The .pt
    holds only tensors, numbers and dicts/lists (loadable with torch.load(weights_only=True))."""
    import shutil
    import tempfile
    from diamond.utils import Checkpointer
    T, N, D, A = 8, 16, 4, 2
    cfg = diamond.PPOConfig(rollout_steps=T, num_envs=N, verbose=False)
    env_fn = lambda: gym_stub.SyntheticEnv(D, A)
    rng = np.random.default_rng(2024)
    a1 = diamond.PPO(env_fn, cfg=cfg)
    a1.learn(synth_experience(rng, T, N, D, A, False, 0.1, 0.05))
    out = {}
    with tempfile.TemporaryDirectory() as d:
        ck = Checkpointer(folder=d, run_name="golden")
        ck.save(T * N, a1.network, a1.optimizer)
        src = os.path.join(d, f"golden-step{T * N:06d}.pt")
        dst = os.path.join(HERE, "ckpt_cartpole-step000128.pt")
        shutil.copyfile(src, dst)
    a2 = diamond.PPO(env_fn, cfg=cfg)          # fresh agent: its own init, then the checkpoint
    Checkpointer().load(dst, a2.network, a2.optimizer)
    exp = synth_experience(rng, T, N, D, A, False, 0.1, 0.05)
    for i, k in enumerate(("obs", "next_obs", "actions", "rewards", "term", "trunc")):
        out[f"exp/{k}"] = np.asarray([row[i] for row in exp])
    st = np.random.get_state()
    out["rng_state"] = np.array(st[1])
    out["rng_pos"] = np.array(st[2])
    losses = []
    real_backward = torch.Tensor.backward

    def backward_wrap(self, *a, **k):
        losses.append(float(self.detach()))
        return real_backward(self, *a, **k)

    torch.Tensor.backward = backward_wrap
    try:
        a2.learn(exp)
    finally:
        torch.Tensor.backward = real_backward
    out["loss"] = np.array(losses)
    out["param_names"] = np.array([n for n, _ in a2.network.named_parameters()])
    for n, p in a2.network.named_parameters():
        out[f"final/{n}"] = p.detach().numpy().copy()
    for n, p in a2.network.named_parameters():
        stt = a2.optimizer.state[p]
        out[f"adam/{n}/exp_avg"] = stt["exp_avg"].numpy().copy()
        out[f"adam/{n}/step"] = np.array(float(stt["step"]))
    np.savez_compressed(os.path.join(HERE, "ckpt_cartpole_resume.npz"), **out)
    print("ckpt_cartpole-step000128.pt + ckpt_cartpole_resume.npz:", len(losses), "steps after load")


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference not present; fixtures are generated only in the survey container")
    torch.set_num_threads(8)
    gym_stub, diamond, ref_ppo, ref_cppo = _import_reference()
    if sys.argv[1:] == ["checkpoint"]:
        make_checkpoint_fixture(diamond, gym_stub)
        return
    if sys.argv[1:] == ["c1"]:
        make_c1_trace(diamond, gym_stub)
        return
    make_checkpoint_fixture(diamond, gym_stub)
    make_perm_golden()
    make_gae_cases(diamond, gym_stub)
    make_learn_trace(diamond, gym_stub, "cartpole_small", continuous=False, T=8, N=16, D=4, A=2,
                     n_learn=2)
    make_learn_trace(diamond, gym_stub, "cartpole_decay", continuous=False, T=8, N=16, D=4, A=2,
                     n_learn=2, cfg_over=dict(decay_lr=True, total_steps=8 * 16 * 3))
    make_learn_trace(diamond, gym_stub, "lunar_medium", continuous=False, T=32, N=64, D=8, A=4,
                     p_term=0.02, p_trunc=0.005, save_all_grads=False)
    make_learn_trace(diamond, gym_stub, "lunar_noadvnorm", continuous=False, T=16, N=32, D=8, A=4,
                     cfg_over=dict(advantage_norm=False, num_minibatches=4, num_epochs=2,
                                   ppo_clip=0.1, entropy_beta=0.05, value_loss_weight=0.5),
                     save_all_grads=False)
    make_learn_trace(diamond, gym_stub, "cheetah_small", continuous=True, T=8, N=16, D=17, A=6,
                     n_learn=2, p_term=0.0, p_trunc=0.05)
    make_learn_trace(diamond, gym_stub, "pendulum_medium", continuous=True, T=32, N=32, D=3, A=1,
                     p_term=0.0, p_trunc=0.01, save_all_grads=False)
    make_c1_trace(diamond, gym_stub)


def make_c1_trace(diamond, gym_stub):
    """BASELINE configs[0] at its own size: CartPole PPO, T=128 x N=8 (B=1,024, minibatches of
    128), the reference's defaults otherwise (ppo.py:15-37), SURVEY 8(d) done rates; two learn()
    calls (Adam and RNG continuation)."""
    make_learn_trace(diamond, gym_stub, "cartpole_c1", continuous=False, T=128, N=8, D=4, A=2,
                     n_learn=2, p_term=0.02, p_trunc=0.005)


if __name__ == "__main__":
    main()
