"""Device Fisher-Yates resolution alone (dppo_perm_resolve) on configs[4]-sized swap targets
(4 epochs x 8,388,608 by default): mean time per call by HIP events, and (unless --no-check)
the result against np.random.permutation.  DPPO_LIB selects the library (timing-only scatter
ablations of csrc/shuffle.hip return after the scatter: run them with --no-check, never in a
learn).  Run under rocprofv3 --kernel-trace --stats for the per-pass split."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "diamond-ppo_amd"))
from diamond import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8388608)
    ap.add_argument("--count", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--walk", default="0")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--public", action="store_true",
                    help="the public 3 * count * n scratch (default: dppo_perm_resolve_scratch)")
    a = ap.parse_args()
    os.environ["DPPO_PERM_WALK"] = a.walk
    n, count = a.n, a.count
    np.random.seed(123)
    key, pos, _ = N.mt_state()
    tg = np.empty(count * n, np.int32)
    N.perm_targets_numpy(key, pos, n, count, tg)
    dev = torch.device("cuda:0")
    td = torch.from_numpy(tg).to(dev)
    out = torch.empty(count * n, dtype=torch.int32, device=dev)
    ints = 3 * count * n if a.public else N.perm_resolve_scratch(n, count)
    scratch = torch.empty(ints, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    call = lambda: N.perm_resolve_ex(td.data_ptr(), out.data_ptr(), n, count, scratch.data_ptr(),
                                     ints, st)
    for _ in range(3):
        call()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        call()
    e1.record()
    torch.cuda.synchronize(dev)
    res = {"n": n, "count": count, "walk": a.walk, "scratch_ints": ints,
           "lib": os.environ.get("DPPO_LIB", "default"),
           "ms_per_call": round(e0.elapsed_time(e1) / a.reps, 4)}
    if not a.no_check:
        np.random.seed(123)
        ref = np.concatenate([np.random.permutation(n) for _ in range(count)]).astype(np.int32)
        res["bit_exact"] = bool(np.array_equal(out.cpu().numpy(), ref))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
