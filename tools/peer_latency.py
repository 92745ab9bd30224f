#!/usr/bin/env python3
"""Latency of the peer exchange (csrc/peer.hip) between `world` processes sharing GPU 0:
    python tools/peer_latency.py [world]
Prints the microseconds per gradient-sized exchange measured by each rank (200 back to back),
using tests/dist_scripts/peer_dp.py's "handle" job (which also checks a learn on each rank
against the world-1 learn).  DPPO_LIB selects the library build."""
import multiprocessing as mp
import os
import socket
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from dist_scripts import peer_dp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        outs = [os.path.join(d, f"r{r}.npz") for r in range(world)]
        ps = [ctx.Process(target=peer_dp.run, args=(r, world, port, "handle", outs[r]))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(200)
        assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
        us = [float(np.load(o)["us_per_exchange"]) for o in outs]
    print(f"lib={os.environ.get('DPPO_LIB', 'default')} world={world} us_per_exchange=" +
          " ".join(f"{u:.2f}" for u in us), flush=True)


if __name__ == "__main__":
    main()
