#!/usr/bin/env python3
"""Variants of the GAE launch's data movement (tools/probe/stream_probe2.hip) at T = 128 and
N (default 8192) over 16 rotating buffer sets; run under rocprofv3 --kernel-trace --stats for the
per-variant kernel durations (stream2_kernel<MODE>).  Grids: 256 x {1,2,4} and the default 1024.

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/probe/stream_probe2.hip \
        -o tools/probe/libstream_probe2.so
    python tools/probe/stream_probe2.py [N]"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libstream_probe2.so"))
lib.probe_stream2.argtypes = [ctypes.c_void_p] * 7 + [ctypes.c_int64, ctypes.c_int,
                                                      ctypes.c_void_p, ctypes.c_int]
T, N, sets = 128, int(sys.argv[1]) if len(sys.argv) > 1 else 8192, 16
dev = torch.device("cuda", 0)
bufs = [[torch.randn(T, N, device=dev), torch.zeros(T, N, dtype=torch.uint8, device=dev),
         torch.zeros(T, N, dtype=torch.uint8, device=dev), torch.randn(T, N, device=dev),
         torch.randn(T, N, device=dev), torch.empty(T, N, device=dev),
         torch.empty(T, N, device=dev)] for _ in range(sets)]
s = torch.cuda.current_stream().cuda_stream
for mode in range(8):
    for grid in ((256, 512, 1024) if not (mode & 2) else (256, 512)):
        for rep in range(4):
            for b in bufs:
                assert lib.probe_stream2(*[x.data_ptr() for x in b], T * N, grid, s, mode) == 0
        torch.cuda.synchronize()
print("done", flush=True)
