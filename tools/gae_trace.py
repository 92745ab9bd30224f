#!/usr/bin/env python3
"""Hand-off timeline of the pipelined GAE kernel (timing-only build).

    make -C diamond-ppo_amd variant-gae NAME=gtrace DEFS=-DDPPO_GAE_TRACE
    DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so python tools/gae_trace.py [--N 8192]

Runs the GAE over rotating buffer sets (as tools/gae_bench.py), then prints, for workgroups 0 and
128 of the last launch, s_memtime cycles (relative to the workgroup's start stamp) at which each
chunk owner's loads had landed, its scan wait ended and its stores were issued, and at which the
scan saw / finished each chunk.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
from diamond import _native as NN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--N", type=int, default=8192)
    ap.add_argument("--sets", type=int, default=16)
    ap.add_argument("--affine", action="store_true", help="the affine-scan kernel's timeline")
    a = ap.parse_args()
    T, N = a.T, a.N
    dev = torch.device("cuda", 0)
    h = NN.Handle(0, NN.Dims(T, N, 1, 1, 0, 64, 1, 1, 1, 0))
    if a.affine:
        h.set_gae_mode(NN.GAE_AFFINE)
    rng = np.random.default_rng(1)
    g = lambda x: torch.from_numpy(x).to(dev)
    bufs = [[g(rng.normal(1, 1, (T, N)).astype(np.float32)),
             g((rng.random((T, N)) < 0.02).astype(np.uint8)),
             g((rng.random((T, N)) < 0.005).astype(np.uint8)),
             g(rng.standard_normal((T, N), dtype=np.float32)),
             g(rng.standard_normal((T, N), dtype=np.float32)),
             torch.empty(T, N, device=dev), torch.empty(T, N, device=dev)] for _ in range(a.sets)]
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        for b in bufs:
            NN.check(h.lib.dppo_gae_f32(h.h, *[x.data_ptr() for x in b], 0.99, 0.95, s))
    torch.cuda.synchronize()
    buf = np.zeros((2, 48), np.int64)
    fn = h.lib.dppo_debug_gae_trace
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    for w in range(2):
        t = buf[w] - buf[w][0]
        print(f"workgroup {0 if w == 0 else 128}: end {t[41]} cycles")
        if a.affine:
            print("  chunk  loads-landed  map-published  later-maps-seen  fold-done  "
                  "stores-issued")
            for k in range(7, -1, -1):
                print(f"  {k:5d}  {t[1 + k]:12d}  {t[9 + k]:15d}  {t[25 + k]:14d}  "
                      f"{t[33 + k]:9d}  {t[17 + k]:13d}")
            continue
        print("  chunk  loads-landed  scan-seen  scan-done  owner-wait-done  stores-issued")
        for k in range(7, -1, -1):
            print(f"  {k:5d}  {t[1 + k]:12d}  {t[25 + k]:9d}  {t[33 + k]:9d}  {t[9 + k]:15d}  "
                  f"{t[17 + k]:13d}")


if __name__ == "__main__":
    main()
