"""The RCCL leg of the data-parallel path executed on a one-GPU box: a 1-rank
torch.distributed.run job whose agents hold a real RCCL communicator (DPPO_FORCE_COMM=1), so
ncclCommInitRank, the advantage-stat and per-minibatch gradient ncclAllReduce calls and the
slab_reduce -> all-reduce -> clip_adam sequence all run, and reproduce the reference traces
(tests/dist_scripts/rccl_one_rank.py).  RCCL refuses two ranks on one device, so more ranks are
covered by the loopback group (test_gpu_dataparallel.py) and the gloo tests."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_rccl_one_rank_learn_matches_reference_traces():
    script = os.path.join(ROOT, "tests", "dist_scripts", "rccl_one_rank.py")
    env = dict(os.environ, DPPO_FORCE_COMM="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               MASTER_ADDR="127.0.0.1")
    env.pop("DPPO_SPLIT_ADAM", None)
    env.pop("DPPO_FUSED_ADAM", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    out = r.stdout + "\n" + r.stderr
    print(out[-4000:])
    assert r.returncode == 0, out[-6000:]
    assert "RCCL_ONE_RANK_OK" in r.stdout
