#!/usr/bin/env python3
"""Data-movement ceiling of the GAE's 22 B/element at T x N in one launch (no recurrence):
tools/probe/stream_probe.hip over rotating buffer sets, per-launch time from one event pair around
a sweep.  Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/probe/stream_probe.hip -o
tools/probe/libstream_probe.so"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libstream_probe.so"))
lib.probe_stream.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                            ctypes.c_int]
T, N, sets = 128, int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 16
dev = torch.device("cuda", 0)
bufs = [[torch.randn(T, N, device=dev), torch.zeros(T, N, dtype=torch.uint8, device=dev),
         torch.zeros(T, N, dtype=torch.uint8, device=dev), torch.randn(T, N, device=dev),
         torch.randn(T, N, device=dev), torch.empty(T, N, device=dev),
         torch.empty(T, N, device=dev)] for _ in range(sets)]
s = torch.cuda.current_stream().cuda_stream
for wt in (0, 1):
  for grid in (256, 512, 1024, 2048, 4096):
    for b in bufs:
        lib.probe_stream(*[x.data_ptr() for x in b], T * N, grid, s, wt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        for b in bufs:
            lib.probe_stream(*[x.data_ptr() for x in b], T * N, grid, s, wt)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (4 * sets)
    print(json.dumps({"N": N, "grid": grid, "write_through": wt,
                      "us_per_launch_in_sweep": round(us, 2),
                      "GBps": round(22 * T * N / us / 1e3, 1)}), flush=True)
