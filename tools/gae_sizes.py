#!/usr/bin/env python3
"""GAE roofline evidence at N = 8192 and N = 65,536 (C5's one-GPU buffer): the bit-exact serial
kernel, the affine-scan kernel and the no-recurrence streaming probe (tools/probe/stream_probe.hip,
same 22 B/element, same rotating sets past the 256 MB Infinity Cache), per-launch times.

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/probe/stream_probe.hip \
        -o tools/probe/libstream_probe.so
    python tools/gae_sizes.py            (run it under rocprofv3 --kernel-trace --stats too)
"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def probe(N, T=128, grid=1024, reps=4):
    lib = ctypes.CDLL(os.path.join(HERE, "probe", "libstream_probe.so"))
    lib.probe_stream.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_int,
                                                         ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    sets = max(2, -(-369 * 2 ** 20 // (22 * T * N)))
    bufs = [[torch.randn(T, N, device=dev), torch.zeros(T, N, dtype=torch.uint8, device=dev),
             torch.zeros(T, N, dtype=torch.uint8, device=dev), torch.randn(T, N, device=dev),
             torch.randn(T, N, device=dev), torch.empty(T, N, device=dev),
             torch.empty(T, N, device=dev)] for _ in range(sets)]
    s = torch.cuda.current_stream().cuda_stream
    for b in bufs:
        lib.probe_stream(*[x.data_ptr() for x in b], T * N, grid, s, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for b in bufs:
            lib.probe_stream(*[x.data_ptr() for x in b], T * N, grid, s, 0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * sets)
    del bufs
    torch.cuda.empty_cache()
    return {"us_per_launch_in_sweep": round(us, 2), "GBps": round(22 * T * N / us / 1e3, 1),
            "frac": round(22 * T * N / us / 1e3 / bench.HBM_PEAK_GBS, 4), "grid": grid,
            "rotating_sets": sets}


def main():
    dev = torch.device("cuda", 0)
    for N in (8192, 65536):
        out = {"N": N}
        if os.path.exists(os.path.join(HERE, "probe", "libstream_probe.so")):
            out["probe"] = probe(N)
        for mode, name in ((0, "exact"), (1, "affine")):
            r = bench.gae_roofline(dev, N=N, mode=mode)
            out[name] = {k: r[k] for k in ("us_per_launch", "achieved", "frac", "rotating_sets",
                                           "launches")}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
