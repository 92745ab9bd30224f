#!/usr/bin/env python3
"""GAE kernel micro-benchmark: dppo_gae_f32 at T x N over `sets` rotating buffer sets (more bytes
than the 256 MB Infinity Cache), timed (a) with a HIP event pair around every launch and (b) as one
event pair around a whole sweep of back-to-back launches.  Run it under
`rocprofv3 --kernel-trace --stats` for the kernel durations themselves.

    python tools/gae_bench.py [--T 128] [--N 8192] [--sets 16] [--reps 8]
"""
import argparse
import json
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
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--affine", action="store_true", help="the affine-scan (tolerance) mode")
    ap.add_argument("--with-probe", action="store_true",
                    help="after every GAE sweep, the same sweep of dppo_gae_stream_probe (the "
                         "no-recurrence ceiling over the same buffers)")
    a = ap.parse_args()
    T, N = a.T, a.N
    dev = torch.device("cuda", 0)
    h = NN.Handle(0, NN.Dims(T, N, 1, 1, 0, 64, 1, 1, 1, 0))
    if a.affine:
        h.set_gae_mode(NN.GAE_AFFINE)
    rng = np.random.default_rng(1)
    bufs = []
    for _ in range(a.sets):
        g = lambda x: torch.from_numpy(x).to(dev)
        bufs.append([g(rng.normal(1, 1, (T, N)).astype(np.float32)),
                     g((rng.random((T, N)) < 0.02).astype(np.uint8)),
                     g((rng.random((T, N)) < 0.005).astype(np.uint8)),
                     g(rng.standard_normal((T, N), dtype=np.float32)),
                     g(rng.standard_normal((T, N), dtype=np.float32)),
                     torch.empty(T, N, device=dev), torch.empty(T, N, device=dev)])
    s = torch.cuda.current_stream(dev)

    def launch(b):
        NN.check(h.lib.dppo_gae_f32(h.h, *[x.data_ptr() for x in b], 0.99, 0.95, s.cuda_stream))

    for b in bufs:
        launch(b)
    torch.cuda.synchronize()
    per = []
    for _ in range(a.reps):
        for b in bufs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch(b)
            e1.record(s)
            per.append((e0, e1))
    torch.cuda.synchronize()
    per_ms = np.array([x.elapsed_time(y) for x, y in per])
    sweeps = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for b in bufs:
            launch(b)
        e1.record(s)
        sweeps.append((e0, e1))
    torch.cuda.synchronize()
    sw_ms = np.array([x.elapsed_time(y) for x, y in sweeps]) / a.sets
    def probe(b):
        NN.check(h.lib.dppo_gae_stream_probe(h.h, *[x.data_ptr() for x in b], s.cuda_stream),
                 "dppo_gae_stream_probe")

    h.set_timing(True)
    for _ in range(a.reps):
        for b in bufs:
            launch(b)
        if a.with_probe:
            for b in bufs:
                probe(b)
    tm = h.timing()
    kms, kcnt = tm["gae"]
    h.set_timing(False)
    nbytes = 22 * T * N
    out = {"T": T, "N": N, "staged": bool(os.environ.get("DPPO_GAE_STAGED")),
           "us_event_pair_median": round(float(np.median(per_ms)) * 1e3, 2),
           "us_event_pair_min": round(float(per_ms.min()) * 1e3, 2),
           "us_per_launch_in_sweep": round(float(np.median(sw_ms)) * 1e3, 2),
           "us_kernel_events": round(kms / kcnt * 1e3, 2),
           "GBps_kernel_events": round(nbytes / (kms / kcnt * 1e-3) / 1e9, 1),
           "GBps_event_pair": round(nbytes / (np.median(per_ms) * 1e-3) / 1e9, 1),
           "GBps_sweep": round(nbytes / (np.median(sw_ms) * 1e-3) / 1e9, 1)}
    if a.with_probe:
        pms, pcnt = tm["gae_probe"]
        out["us_probe_kernel_events"] = round(pms / pcnt * 1e3, 2)
        out["frac_of_ceiling"] = round(pms / pcnt / (kms / kcnt), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
