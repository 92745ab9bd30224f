"""RecurrentPPO under data parallelism (reference recurrent_ppo.py:301-367, which
itself crashes at :78, so the yardstick is this build's own single-process learn()).

Two processes in a gloo group, both on the one GPU, each learn() on half of the env axis of one
rollout (num_minibatches = 1, the reference default: every epoch's minibatch is the whole
batch).  With the global advantage statistics, the 1/world loss scaling and the gradient
all-reduce, both ranks must end with the parameters of one process that learned on the whole
env axis (up to the re-association of the sums), and with identical parameters to each other."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_recurrent_ppo_two_ranks_match_one(tmp_path):
    from dist_scripts import recurrent_dp
    T, Ng, D, A = 16, 16, 5, 3
    ctx = mp.get_context("spawn")
    outs = {}
    for world in (1, 2):
        port = _free_port()
        procs = []
        for r in range(world):
            path = str(tmp_path / f"w{world}_r{r}.npz")
            outs[(world, r)] = path
            procs.append(ctx.Process(target=recurrent_dp.run,
                                     args=(r, world, port, T, Ng, D, A, path)))
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    one = np.load(outs[(1, 0)])
    r0, r1 = np.load(outs[(2, 0)]), np.load(outs[(2, 1)])
    assert np.array_equal(r0["init"], one["init"]) and np.array_equal(r1["init"], one["init"])
    assert np.array_equal(r0["final"], r1["final"])      # replicated clip + Adam on one gradient
    assert np.all(np.isfinite(r0["final"]))
    moved = np.abs(one["final"] - one["init"])
    assert moved.max() > 1e-4                            # 3 Adam steps of lr 3e-4 were taken
    # the two-rank sums re-associate the one-rank ones (gradients equal to ~1e-6 relative); over
    # three Adam steps of ~lr * sign(g) that stays far below lr
    np.testing.assert_allclose(r0["final"], one["final"], rtol=0, atol=2e-5)
