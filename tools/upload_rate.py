#!/usr/bin/env python3
"""The per-rank upload of the reference-exact mode at BASELINE configs[4], measured on one GPU.

With global minibatches every rank uploads all E x T x 65,536 Fisher-Yates targets per learn
(4 x 8.4 M int32 = 134 MB: the bucket build needs every target) from the node-shared
draft slot in /dev/shm (hipHostRegister'ed, drawshare.py) on the handle's copy stream
(capi.cpp upload_perms), which starts once the learn two back has released the device slot, so
in a device-bound run it overlaps the previous learn.  `gmb_cap.py` models a learn at world 8 as
max(draw, device); this tool measures the third term on one MI355X:

* the H2D time of 134 MB from torch-pinned memory and from a registered POSIX shared-memory
  segment (the drawshare path), HIP events on the copy's own stream, median of reps;
* whether those copies slow the device: world-8 share learns of configs[4] (8,192 envs, the
  rank's local share) timed alone, with one 134 MB upload issued on its own stream as each learn
  is enqueued (each gated on the previous one, as the draft slots are: the global mode's cadence),
  and with uploads kept running back to back by a side thread (the copy engine saturated).  Every
  MI355X has its own PCIe link, so one GPU with one stream of uploads is one rank's situation on
  the node, except for the host memory the 8 ranks' reads share.

    python tools/upload_rate.py [--out file.json]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))

NBYTES = 4 * 128 * 65536 * 4  # E x T x 65,536 int32 targets


def hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    lib.hipHostUnregister.argtypes = [ctypes.c_void_p]
    lib.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    return lib


def copy_ms(lib, dst, src_ptr, stream, reps=9):
    import torch
    ts = []
    for r in range(reps + 1):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        assert lib.hipMemcpyAsync(dst.data_ptr(), src_ptr, NBYTES, 1, stream.cuda_stream) == 0
        b.record(stream)
        b.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def share8_agent(dev):
    """One rank's share of configs[4] at world 8 (8,192 CartPole-shaped envs), device rollout."""
    import bench
    import diamond
    cfg = diamond.PPOConfig(rollout_steps=128, num_envs=8192, verbose=False, total_steps=10 ** 12)
    agent = diamond.PPO(None, cfg, envs=bench.SpecEnvs(4, 2, False))
    ro, _ = bench.synth_rollout(128, 8192, 4, 2, False, 0.02, 0.005, seed=0, device=dev)
    for _ in range(3):
        agent.learn_device(ro)
    return agent, ro


def timed(agent, ro, steps, dev, before=None):
    """ms per learn over `steps` learns; `before()` runs ahead of each learn's enqueue."""
    import torch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        if before is not None:
            before()
        agent.learn_device(ro)
    torch.cuda.synchronize(dev)
    return round((time.perf_counter() - t0) / steps * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from multiprocessing import shared_memory
    dev = torch.device("cuda", 0)
    lib = hip()
    dst = torch.empty(NBYTES // 4, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    pinned = torch.from_numpy(np.arange(NBYTES // 4, dtype=np.int32)).pin_memory()
    res = {"bytes": NBYTES}
    res["pinned_ms"] = copy_ms(lib, dst, pinned.data_ptr(), side)
    shm = shared_memory.SharedMemory(create=True, size=NBYTES)
    try:
        view = np.ndarray((NBYTES // 4,), np.int32, buffer=shm.buf)
        view[:] = 7
        ptr = view.ctypes.data
        assert lib.hipHostRegister(ptr, NBYTES, 0) == 0, "hipHostRegister failed"
        try:
            res["shm_registered_ms"] = copy_ms(lib, dst, ptr, side)
            res["shm_registered_GBps"] = round(NBYTES / res["shm_registered_ms"] / 1e6, 1)
            torch.cuda.synchronize(dev)
            assert int(dst[-1].item()) == 7

            agent, ro = share8_agent(dev)
            dst2 = [dst, torch.empty_like(dst)]
            done = [torch.cuda.Event(), torch.cuda.Event()]
            for ev in done:
                ev.record(side)
            nxt = [0]

            def per_learn():
                """One upload per learn into alternating device buffers, each gated on the upload
                two back (the engine's double-buffered device slots, capi.cpp upload_perms)."""
                k = nxt[0] & 1
                nxt[0] += 1
                done[k].synchronize()
                assert lib.hipMemcpyAsync(dst2[k].data_ptr(), ptr, NBYTES, 1,
                                          side.cuda_stream) == 0
                done[k].record(side)

            stop = threading.Event()
            uploads = [0]

            def pump():  # back to back, from a side thread
                while not stop.is_set():
                    lib.hipMemcpyAsync(dst.data_ptr(), ptr, NBYTES, 1, side.cuda_stream)
                    side.synchronize()
                    uploads[0] += 1

            rows = {"alone": [], "one_upload_per_learn": [], "uploads_back_to_back": []}
            for _ in range(a.reps):  # interleaved
                rows["alone"].append(timed(agent, ro, a.steps, dev))
                rows["one_upload_per_learn"].append(timed(agent, ro, a.steps, dev, per_learn))
                side.synchronize()
                uploads[0] = 0
                th = threading.Thread(target=pump, daemon=True)
                th.start()
                t0 = time.perf_counter()
                rows["uploads_back_to_back"].append(timed(agent, ro, a.steps, dev))
                el = time.perf_counter() - t0
                stop.set()
                th.join()
                stop.clear()
                res.setdefault("uploads_per_s_back_to_back", []).append(round(uploads[0] / el, 1))
            res["share8_ms_per_learn"] = rows
        finally:
            lib.hipHostUnregister(ptr)
    finally:
        shm.close()
        shm.unlink()
    res["pinned_ms"] = round(res["pinned_ms"], 3)
    res["shm_registered_ms"] = round(res["shm_registered_ms"], 3)
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
