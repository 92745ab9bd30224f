"""engine.NativeLearner._init_comm on a world-2 gloo group (CPU; the handle is a stand-in): the
ranks agree on the transport of the data-parallel exchange.  Under DPPO_COMM=auto a failing
peer-exchange self-test on ONE rank makes EVERY rank close the peer exchange, warn, and keep the
RCCL communicator; under DPPO_COMM=peer the same failure raises on every rank; a rank that cannot
map a peer buffer takes the others down the same path.  (The GPU side of the same path --
a real self-test, a peer that stops exchanging -- is tests/test_gpu_peer.py.)"""
import os
import socket
import warnings

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeHandle:
    def __init__(self, rank, fail_open, fail_test):
        self.rank, self.fail_open, self.fail_test = rank, fail_open, fail_test
        self.calls = []

    def comm_init(self, nranks, rank, uid):
        self.calls.append("comm_init")

    def peer_export(self):
        return bytes([self.rank]) * 64

    def peer_open(self, nranks, rank, handles, shared_device=False):
        self.calls.append("peer_open")
        assert len(handles) == 64 * nranks and not shared_device
        return "cannot map" if self.fail_open else ""

    def peer_selftest(self, stream):
        self.calls.append("peer_selftest")
        return "element 3 is 7, expected 6" if self.fail_test else ""

    def peer_close(self):
        self.calls.append("peer_close")


class _FakeFlat:
    def __init__(self):
        self.flat = torch.zeros(8)


class _CurrentStream:
    cuda_stream = 0


def _worker(rank, world, port, mode, fail_open_rank, fail_test_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPPO_COMM=mode)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "diamond-ppo_amd"))
    from diamond import engine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        engine.N.comm_unique_id = lambda: bytes(128)
        torch.cuda.current_stream = lambda device=None: _CurrentStream()
        L = object.__new__(engine.NativeLearner)
        L.world, L.rank, L.device = world, rank, torch.device("cpu")
        L.handle = _FakeHandle(rank, rank == fail_open_rank, rank == fail_test_rank)
        L.flat = _FakeFlat()
        L._gpu_identity = lambda: ("host", 0, rank, 0)   # distinct GPUs
        err = ""
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            try:
                L._init_comm()
            except RuntimeError as e:
                err = str(e)
        q.put((rank, getattr(L, "peer", None), L.handle.calls, err,
               [str(x.message) for x in w]))
    finally:
        dist.destroy_process_group()


def _run(mode, fail_open_rank=-1, fail_test_rank=-1):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, fail_open_rank,
                                                fail_test_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, peer, calls, err, warns = q.get(timeout=120)
        res[r] = {"peer": peer, "calls": calls, "err": err, "warns": warns}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(300)
def test_auto_all_ranks_pass_selftest_use_peer():
    res = _run("auto")
    for r in (0, 1):
        assert res[r]["peer"] is True and not res[r]["err"] and not res[r]["warns"]
        assert res[r]["calls"] == ["comm_init", "peer_open", "peer_selftest"]


@pytest.mark.timeout(300)
def test_auto_one_rank_fails_selftest_every_rank_falls_back_to_rccl():
    res = _run("auto", fail_test_rank=1)
    for r in (0, 1):
        assert res[r]["peer"] is False and not res[r]["err"]
        assert res[r]["calls"] == ["comm_init", "peer_open", "peer_selftest", "peer_close"]
        assert any("RCCL carries the exchange" in m for m in res[r]["warns"]), res[r]["warns"]
    assert "expected 6" in " ".join(res[1]["warns"])
    assert "another rank failed" in " ".join(res[0]["warns"])


@pytest.mark.timeout(300)
def test_auto_one_rank_cannot_map_every_rank_falls_back():
    res = _run("auto", fail_open_rank=0)
    for r in (0, 1):
        assert res[r]["peer"] is False and "peer_selftest" not in res[r]["calls"]
        assert any("RCCL carries the exchange" in m for m in res[r]["warns"])
    assert res[1]["calls"][-1] == "peer_close"      # rank 1 had mapped: it unmaps


@pytest.mark.timeout(300)
def test_peer_required_failure_raises_on_every_rank():
    res = _run("peer", fail_test_rank=0)
    for r in (0, 1):
        assert "peer exchange unavailable" in res[r]["err"]
        assert "comm_init" not in res[r]["calls"]
