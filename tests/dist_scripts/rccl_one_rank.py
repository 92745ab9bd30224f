"""Run under ``torch.distributed.run --nproc-per-node 1`` with DPPO_FORCE_COMM=1 (launched by
tests/test_gpu_rccl.py): the drop-in agents build their libdppo handle with a 1-rank RCCL
communicator bootstrapped through engine._init_comm (unique id broadcast over the torch "nccl"
process group), so every learn() runs the collective sequence -- advantage-stat ncclAllReduce,
then per minibatch slab_reduce_kernel -> ncclAllReduce -> clip_adam_kernel -- and must reproduce
the reference's captured learn() traces.  Prints RCCL_ONE_RANK_OK and exits 0 on success.
Test infrastructure only."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "diamond-ppo_amd"), ROOT, os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    assert os.environ.get("DPPO_FORCE_COMM") == "1"
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl")
    assert dist.get_world_size() == 1
    import diamond
    from conftest import load_golden
    from test_gpu_parity import experience, make_agent

    for name in ("cartpole_c1", "cartpole_small", "cheetah_small"):
        z = load_golden(f"learn_{name}.npz")
        T, Nn, D, A, cont, n_learn = (int(x) for x in z["dims"])
        agent = make_agent(z)
        L = agent._learner
        assert L.fused and L.world == 1
        L.handle.set_timing(True)
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
        tm = L.handle.timing()
        E, M = int(z["cfg/num_epochs"]), int(z["cfg/num_minibatches"])
        # one gradient all-reduce per minibatch + one advantage-stat all-reduce per learn, and
        # the split kernels, not reduce_adam, after them
        assert tm["allreduce"][1] == n_learn * (E * M + 1), tm
        assert tm["clip_adam"][1] == n_learn * E * M and tm["reduce_adam"][1] == 0, tm
        np.testing.assert_allclose(losses, z["loss"], rtol=2e-5, atol=2e-5, err_msg=name)
        np.testing.assert_allclose(norms, z["norm"], rtol=2e-5, atol=2e-5, err_msg=name)
        for n, p in agent.network.named_parameters():
            np.testing.assert_allclose(p.detach().cpu().numpy(), z["final/" + n], rtol=0,
                                       atol=5e-6, err_msg=f"{name} {n}")
        print(f"{name}: {len(losses)} steps through RCCL, {tm['allreduce'][1]} all-reduces, "
              f"{tm['allreduce'][0]:.3f} ms", flush=True)
        L.close()
    dist.destroy_process_group()
    print("RCCL_ONE_RANK_OK", flush=True)


if __name__ == "__main__":
    main()
