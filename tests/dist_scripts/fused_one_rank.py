"""One variant of the 1-rank fused peer exchange (tests/test_gpu_peer.py), run in a process of its
own: the exchange buffer's memory type is a per-process choice (one type per process: csrc/capi.cpp
dppo_peer_export), so each memory type gets a fresh process.  run() writes
"ok" or the failure's traceback to `out_path`.  Test infrastructure only."""
import os
import sys
import traceback


def _paths():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for p in (os.path.join(root, "diamond-ppo_amd"), root, os.path.join(root, "tests"),
              os.path.join(root, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)


def fused_step(variant):
    """Every learn() of the golden cartpole / cheetah traces through a 1-rank peer exchange
    (advantage statistics through the exchange kernel, each minibatch's gradient exchange inside
    reduce_adam_kernel) reproduces the reference's captured traces."""
    import numpy as np
    import torch
    import diamond
    from conftest import load_golden
    from gpu_helpers import stream
    from test_gpu_parity import experience, make_agent
    for name in ("cartpole_small", "cheetah_small"):
        z = load_golden(f"learn_{name}.npz")
        T, Nn, D, A, cont, n_learn = (int(x) for x in z["dims"])
        agent = make_agent(z)
        L = agent._learner
        h = L.handle
        assert not h.peer_open(1, 0, h.peer_export())
        err = h.peer_selftest(stream())
        assert not err, err
        info = h.peer_info()
        assert info["ranks"] == 1 and info["fused"], info
        assert info["memory"] == {"coarse": "coarse-grained", "fine": "fine-grained"}.get(
            variant, "uncached"), info
        seq0 = info["exchanges"]
        h.set_timing(True)
        losses, norms = [], []
        for li in range(n_learn):
            np.random.set_state(("MT19937", z[f"rng_state_before{li}"].astype(np.uint32),
                                 int(z[f"rng_pos_before{li}"]), 0, 0.0))
            ro = diamond.engine.stage_experience(experience(z, li), agent.device, bool(cont))
            agent.learn_device(ro)
            tr = agent.learn_trace()
            losses += list(tr[:, 0])
            norms += list(tr[:, 4])
        torch.cuda.synchronize()
        tm = h.timing()
        E, M = int(z["cfg/num_epochs"]), int(z["cfg/num_minibatches"])
        assert tm["allreduce"][1] == n_learn, tm                 # advantage statistics only
        assert tm["reduce_adam"][1] == n_learn * E * M and tm["clip_adam"][1] == 0, tm
        if variant == "wrap":  # the fused exchanges crossed the wrap (0 is skipped)
            assert seq0 >= 0xFFFFFFF0 and h.peer_info()["exchanges"] < seq0, (seq0, h.peer_info())
        np.testing.assert_allclose(losses, z["loss"], rtol=2e-5, atol=2e-5, err_msg=name)
        np.testing.assert_allclose(norms, z["norm"], rtol=2e-5, atol=2e-5, err_msg=name)
        for n, p in agent.network.named_parameters():
            np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0,
                                       atol=5e-6, err_msg=f"{name} {n}")
        L.close()


def mixed():
    """A second exchange-buffer memory type in one process is refused, loudly, at export."""
    import diamond
    from conftest import load_golden
    from test_gpu_parity import make_agent
    z = load_golden("learn_cartpole_small.npz")
    os.environ["DPPO_PEER_MEM"] = "uncached"
    a1 = make_agent(z)
    a1._learner.handle.peer_export()
    os.environ["DPPO_PEER_MEM"] = "coarse"
    a2 = make_agent(z)
    try:
        a2._learner.handle.peer_export()
    except NotImplementedError as e:  # DPPO_EUNSUPPORTED
        assert "already created an uncached exchange buffer" in str(e), str(e)
    else:
        raise AssertionError("a coarse-grained exchange buffer after an uncached one was accepted")
    a2._learner.close()
    a1._learner.close()


def run(variant, out_path):
    _paths()
    try:
        if variant in ("coarse", "fine"):
            os.environ["DPPO_PEER_MEM"] = variant
        if variant == "wrap":
            os.environ["DPPO_TEST_HOOKS"] = "1"
            os.environ["DPPO_PEER_XSEQ0"] = str(0xFFFFFFF0)
        if variant == "mixed":
            mixed()
        else:
            fused_step(variant)
        msg = "ok"
    except BaseException:
        msg = traceback.format_exc()
    with open(out_path, "w") as f:
        f.write(msg)
