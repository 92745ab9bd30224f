#!/usr/bin/env python3
"""Does the exchange buffer's memory type of one handle affect the next handle in the same
process?  For each ordering (first, second) of DPPO_PEER_MEM types, in a fresh child process:
handle A (type `first`): export, 1-rank open, self-test (the fused optimizer-step exchange
included), close; then handle B (type `second`): the same.  Prints one line per ordering.

    python tools/probe/peer_mem_reuse.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PAIRS = [("uncached", "coarse"), ("uncached", "uncached"), ("uncached", "fine"),
         ("fine", "coarse"), ("coarse", "coarse"), ("coarse", "uncached"), ("fine", "uncached")]


def child(first, second):
    sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))
    import torch
    from diamond import _native as N
    out = []
    for mem in (first, second):
        os.environ["DPPO_PEER_MEM"] = mem
        h = N.Handle(0, N.Dims(16, 256, 4, 2, 0, 64, 4, 8, 1, 0, 0))
        err = h.peer_open(1, 0, h.peer_export())
        if not err:
            err = h.peer_selftest(torch.cuda.current_stream().cuda_stream)
        info = h.peer_info()
        out.append({"mem": mem, "memory": info["memory"], "fused": info["fused"],
                    "selftest": err or "passed"})
        h.close()
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) == 3:
        child(sys.argv[1], sys.argv[2])
        return
    env = dict(os.environ, DPPO_PEER_TIMEOUT_S="5")
    for a, b in PAIRS:
        r = subprocess.run([sys.executable, __file__, a, b], env=env, capture_output=True,
                           text=True, timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        print(f"{a} -> {b}: rc {r.returncode} {line}", flush=True)


if __name__ == "__main__":
    main()
