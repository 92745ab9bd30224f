"""The peer exchange (csrc/peer.hip): the data-parallel learn's all-reduces as one
kernel per exchange that publishes each rank's vector in its own IPC-exported buffer and sums all
ranks' buffers in rank order.  Two processes share the one GPU of the box (RCCL refuses that; the
peer exchange does not care whether a mapped buffer is on this device or across xGMI), each
driving its own handle (tests/dist_scripts/peer_dp.py):

* the C ABI: exact self-test (f32 and f64), then dppo_learn_f32 on each rank's env shard in both
  minibatch modes -- identical parameters on both ranks, equal to the world-1 learn of the global
  buffer (local mode: with the union permutations) to the re-association tolerance of
  test_gpu_dataparallel.py;
* the drop-in PPO under DPPO_COMM=peer: engine._init_comm maps, self-tests and agrees; one learn
  leaves both ranks with identical parameters."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(kind, tmp_path, world=2, env=None):
    from dist_scripts import peer_dp
    ctx = mp.get_context("spawn")
    port = _free_port()
    outs = [str(tmp_path / f"{kind}_r{r}.npz") for r in range(world)]
    procs = [ctx.Process(target=peer_dp.run, args=(r, world, port, kind, outs[r], env))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [np.load(o) for o in outs]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mem", ["coarse", "fine", "uncached"])
def test_peer_exchange_two_ranks_learn_matches_single_gpu(tmp_path, mem):
    """Two processes on this GPU, each mapping the other's exchange buffer (hipIpc), for every
    exchange-buffer memory type (DPPO_PEER_MEM: hipMalloc, fine-grained, uncached)."""
    r0, r1 = _spawn("handle", tmp_path, env={"DPPO_PEER_MEM": mem})
    print(f"peer exchange, 2 ranks on one GPU: {float(r0['us_per_exchange']):.2f} us per "
          f"gradient-sized exchange (rank 1: {float(r1['us_per_exchange']):.2f})")
    for gmb in (0, 1):
        assert np.array_equal(r0[f"params{gmb}"], r1[f"params{gmb}"]), gmb
        np.testing.assert_allclose(r0[f"trace{gmb}"][:, 0], r0[f"single_trace{gmb}"][:, 0],
                                   rtol=2e-5, atol=2e-6, err_msg=f"loss, gmb={gmb}")
        np.testing.assert_allclose(r0[f"trace{gmb}"][:, 4], r0[f"single_trace{gmb}"][:, 4],
                                   rtol=2e-5, atol=2e-6, err_msg=f"grad norm, gmb={gmb}")
        np.testing.assert_allclose(r0[f"params{gmb}"], r0[f"single{gmb}"], rtol=0, atol=5e-6,
                                   err_msg=f"params, gmb={gmb}")


@pytest.mark.timeout(300)
def test_peer_exchange_across_the_sequence_wrap(tmp_path):
    """The exchange numbers wrap at 2^32 (0 is reserved) and the buffers are double-buffered by
    parity: counting on from 0xFFFFFFF0, the self-test and both learns cross the wrap and must
    still give identical parameters on both ranks, equal to the world-1 learn."""
    r0, r1 = _spawn("handle", tmp_path, env={"DPPO_PEER_XSEQ0": str(0xFFFFFFF0), "DPPO_TEST_HOOKS": "1"})
    for gmb in (0, 1):
        assert np.array_equal(r0[f"params{gmb}"], r1[f"params{gmb}"]), gmb
        np.testing.assert_allclose(r0[f"params{gmb}"], r0[f"single{gmb}"], rtol=0, atol=5e-6)


@pytest.mark.timeout(300)
def test_dead_peer_fails_loudly_within_the_timeout(tmp_path):
    """A rank that stops exchanging (every peer wait is bounded by
    DPPO_PEER_TIMEOUT_S): the surviving rank's learn() raises the peer-timeout error within the
    timeout instead of hanging, later calls on its handle refuse, and both processes exit."""
    r0, _ = _spawn("dead", tmp_path, env={"DPPO_PEER_TIMEOUT_S": "3"})
    err, again = str(r0["err"]), str(r0["again"])
    assert "peer exchange timed out" in err, err
    assert "rank 1's word" in err, err   # the error word names the rank whose word never came
    assert "peer exchange timed out" in again, again
    assert float(r0["elapsed"]) < float(r0["timeout"]) + 10.0, float(r0["elapsed"])


@pytest.mark.timeout(300)
def test_failing_peer_selftest_is_refused_on_every_rank(tmp_path):
    """A self-test whose sums come out wrong on every rank (rank 1 contributes one wrong element:
    DPPO_PEER_SELFTEST_SKEW) -- the ranks agree on the failure and, with the peer exchange
    required (DPPO_COMM=peer), every agent construction raises; under DPPO_COMM=auto the same
    agreement falls back to RCCL (tests/test_comm_agreement_cpu.py: RCCL refuses two ranks on
    this box's one GPU)."""
    rs = _spawn("selftest_fail", tmp_path, env={"DPPO_PEER_SELFTEST_SKEW": "1", "DPPO_TEST_HOOKS": "1"})
    assert "expected" in str(rs[0]["err"]) or "another rank failed" in str(rs[0]["err"])
    for r in rs:
        assert "peer exchange unavailable" in str(r["err"]), str(r["err"])


@pytest.mark.timeout(300)
def test_node_shared_draw_matches_one_draw_per_rank(tmp_path):
    """Global minibatches with host-drawn swap targets: the node-shared draw (rank 0 draws into
    shared memory, rank 1 uploads from it, drawshare.py) gives bit for bit the parameters, traces
    and NumPy state of one draw per rank, and rank 1 did take rank 0's drafts."""
    r0, r1 = _spawn("share", tmp_path, env={"DPPO_PERM_DEVICE": "1",
                                            "DPPO_PERM_SHARE_TIMEOUT_S": "30"})
    for r in (r0, r1):
        assert np.array_equal(r["final_own"], r["final_shared"])
        assert np.array_equal(r["trace_own"], r["trace_shared"])
        assert np.array_equal(r["rng_own"], r["rng_shared"])
    assert np.array_equal(r0["final_shared"], r1["final_shared"])
    shared, own, mismatch, timeout, leader = (int(x) for x in r1["stats"])
    assert leader == 0 and shared >= 7 and own == 0 and timeout == 0, r1["stats"]
    assert int(r0["stats"][4]) == 1 and int(r0["stats"][0]) >= 7, r0["stats"]


@pytest.mark.timeout(300)
def test_peer_exchange_drop_in_agent(tmp_path):
    r0, r1 = _spawn("agent", tmp_path)
    assert np.array_equal(r0["init"], r1["init"])
    assert np.array_equal(r0["final"], r1["final"])
    assert np.all(np.isfinite(r0["final"])) and np.abs(r0["final"] - r0["init"]).max() > 1e-5
    assert np.array_equal(r0["trace"], r1["trace"])


def _one_process(variant, tmp_path):
    from dist_scripts import fused_one_rank
    ctx = mp.get_context("spawn")
    out = str(tmp_path / f"fused_{variant}.txt")
    p = ctx.Process(target=fused_one_rank.run, args=(variant, out))
    p.start()
    p.join(240)
    if p.is_alive():
        p.kill()
    assert p.exitcode == 0, p.exitcode
    msg = open(out).read()
    assert msg == "ok", msg


@pytest.mark.timeout(300)
@pytest.mark.parametrize("variant", ["uncached", "coarse", "fine", "wrap"])
def test_peer_exchange_one_rank_fused_step_reproduces_reference_traces(tmp_path, variant):
    """A 1-rank peer exchange: every learn() then takes the multi-rank sequence of a node with one
    GPU per rank -- the advantage statistics through the exchange kernel, and each minibatch's
    gradient exchange INSIDE reduce_adam_kernel (publish the block's slice, wait for every rank's
    flag, sum in rank order) -- and must reproduce the reference's captured traces
    (tests/dist_scripts/fused_one_rank.py).  (Two ranks sharing this GPU take the unfused
    exchange: their optimizer-step grids could not be resident at once; the test above.)
    Variants: the exchange buffer uncached (the default), coarse- or fine-grained, and the fused
    exchange counting on from just below the 2^32 sequence wrap (test hook).  Each variant runs in
    a process of its own: the memory type is one per process (DESIGN.md §6 round 6 -- a coarse- or
    fine-grained buffer created after two uncached ones in one process lost a store)."""
    _one_process(variant, tmp_path)


@pytest.mark.timeout(300)
def test_peer_exchange_refuses_a_second_memory_type_in_one_process(tmp_path):
    """dppo_peer_export refuses an exchange buffer whose memory type differs from the one this
    process already created (the allocation history that lost a store)."""
    _one_process("mixed", tmp_path)


def _bench_line(cmd, timeout=280):
    import json
    import os
    import subprocess
    from conftest import ROOT
    env = dict(os.environ, DPPO_BENCH_REHEARSE="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(300)
def test_bench_two_rank_rehearsal_line():
    """bench.py's N > 1 path under an explicit launcher (torch.distributed.run, barrier +
    max-over-ranks timing, one JSON line from rank 0) rehearsed on the box's one GPU:
    DPPO_BENCH_REHEARSE=1 puts both ranks on GPU 0 with a gloo group and the peer exchange
    between them."""
    import sys
    d = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                     "--nproc-per-node=2", "--master-addr=127.0.0.1",
                     f"--master-port={_free_port()}", "bench.py", "--gpus", "2", "--steps", "3",
                     "--warmup", "1", "--config", "cartpole4096"])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    assert d["config"]["exchange"] == "peer" and d["config"]["num_envs_total"] == 2 * 4096
    assert d["kernels"]["allreduce"]["launches"] > 0


@pytest.mark.timeout(300)
def test_bench_gpus_flag_starts_the_ranks_itself():
    """``python bench.py --gpus 2`` with no launcher (how the driver may run its scaling
    sweep): bench.py starts the two ranks itself and rank 0's line says n_gpus 2, on the default
    headline workload (LunarLander, 8192 envs per rank)."""
    import sys
    d = _bench_line([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0
    assert d["config"]["name"] == "lunar8192" and d["config"]["num_envs_total"] == 2 * 8192
    assert d["config"]["exchange"] == "peer"
    # every multi-GPU question of the north star from this one invocation: configs[4] strong
    # scaling in both minibatch modes against a world-1 anchor, and the exchange itself
    mg = d["multi_gpu"]
    ex = mg["exchange"]
    assert ex["transport"] == "peer" and ex["peer_selftest"] == "passed"
    assert ex["us_per_exchange_max_over_ranks"] > 0 and ex["memory"] in (
        "coarse-grained", "fine-grained", "uncached")
    for m in ("local", "global"):
        row = mg[f"c5_strong_{m}"]
        assert row["num_envs_per_gpu"] == 65536 // 2 and row["update_steps_per_s"] > 0
        assert row["minibatches"] == ("global" if m == "global" else "local-union")
        assert mg["c5_update_steps_speedup_vs_world1"][m] > 0
    assert mg["c5_strong_global"]["perm_device_ms_per_step"] > 0
    assert mg["c5_world1_anchor"]["update_steps_per_s"] > 0


@pytest.mark.timeout(300)
def test_bench_one_gpu_line_names_its_baseline_config():
    """The N = 1 line (the driver's BENCH line) names which BASELINE config its headline is --
    configs[2] since round 4 -- and carries the roofline of its dominant kernel."""
    import sys
    d = _bench_line([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-extra",
                     "--no-cpu-baseline", "--no-gae-roofline"])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["unit"] == "env-steps/s"
    assert d["config"]["baseline_config"] == "configs[2]"
    assert d["headline"]["name"] == "lunar8192" and d["headline"]["baseline_config"] == "configs[2]"
    r = d["roofline"]
    assert r["bound"] == "mfma" and 0 < r["frac"] < 1 and r["unit"] == "TFLOP/s"
