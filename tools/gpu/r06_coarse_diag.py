#!/usr/bin/env python3
"""Round 6 diagnosis of the coarse/fine exchange-buffer failure: which
history in one process makes a 1-rank fused exchange miss its own tagged word.  Each case runs in
its own process as a sequence of agents (exchange-buffer memory type, golden learn trace,
per-kernel timing on/off); every agent opens a 1-rank exchange, runs the self-test, then the
golden learns, and is closed.  Prints one line per case: each agent's self-test result.

    python tools/gpu/r06_coarse_diag.py            # every case, one subprocess each
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
U, C, F = "uncached", "coarse", "fine"
CP, CH = "cartpole_small", "cheetah_small"
CASES = {  # name: [(memory, golden, mode)]; mode 0 learns, -1 self-test only, 2 kept alive (not
    # closed); "+acq": DPPO_PEER_ACQ=1 (system-scope acquire before every poll of a peer word);
    # "+noipc": DPPO_PEER_NOIPC=1 (the buffers are never exported with hipIpcGetMemHandle);
    # "+nopool": DPPO_PEER_NOPOOL=1 (exchange buffers freed at handle destruction, the round-5
    # behaviour; since round 6 they stay in a process pool and are never freed)
    "uncached cart x2 > coarse +nopool": [(U, CP, 0), (U, CP, 0), (C, CP, 0)],
    "uncached cart x2 > fine +nopool": [(U, CP, 0), (U, CP, 0), (F, CP, 0)],
    "uncached cart x2 > coarse": [(U, CP, 0), (U, CP, 0), (C, CP, 0)],
    "uncached cart x2 > fine": [(U, CP, 0), (U, CP, 0), (F, CP, 0)],
    "uncached cart x3 > coarse": [(U, CP, 0), (U, CP, 0), (U, CP, 0), (C, CP, 0)],
    "test order (timing)": [(U, CP, 1), (U, CH, 1), (C, CP, 1), (C, CH, 1), (F, CP, 1),
                            (F, CH, 1)],
}


def one(case):
    sys.path[:0] = [os.path.join(ROOT, "diamond-ppo_amd"), ROOT, os.path.join(ROOT, "tests"),
                    os.path.join(ROOT, "tests", "golden")]
    import numpy as np
    import torch
    import diamond
    from conftest import load_golden
    from gpu_helpers import stream
    from test_gpu_parity import experience, make_agent
    os.environ["DPPO_TEST_HOOKS"] = "1"  # mixed memory types are refused since round 6 ...
    os.environ["DPPO_PEER_MIX"] = "1"    # ... except under this diagnosis hook
    if case.endswith("+acq"):
        os.environ["DPPO_TEST_HOOKS"] = "1"
        os.environ["DPPO_PEER_ACQ"] = "1"
    if case.endswith("+nopool"):
        os.environ["DPPO_PEER_NOPOOL"] = "1"
    if case.endswith("+noipc"):
        os.environ["DPPO_TEST_HOOKS"] = "1"
        os.environ["DPPO_PEER_NOIPC"] = "1"
    keep = []
    out = []
    for mem, name, timing in CASES[case]:
        os.environ["DPPO_PEER_MEM"] = mem
        z = load_golden(f"learn_{name}.npz")
        cont = int(z["dims"][4])
        agent = make_agent(z)
        L = agent._learner
        h = L.handle
        assert not h.peer_open(1, 0, h.peer_export())
        err = h.peer_selftest(stream())
        info = h.peer_info()
        out.append(f"{mem[0]}{name[:2]}:{'ok' if not err else 'FAIL ' + err}")
        if err:
            break
        if timing == 1:
            h.set_timing(True)
        for li in range(int(z["dims"][5]) if timing >= 0 else 0):
            np.random.set_state(("MT19937", z[f"rng_state_before{li}"].astype(np.uint32),
                                 int(z[f"rng_pos_before{li}"]), 0, 0.0))
            ro = diamond.engine.stage_experience(experience(z, li), agent.device, bool(cont))
            agent.learn_device(ro)
        torch.cuda.synchronize()
        out[-1] += f"(fused={info['fused']})"
        if timing == 2:
            keep.append(agent)
        else:
            L.close()
    print(f"RESULT {case}: " + " | ".join(out), flush=True)


def main():
    if len(sys.argv) > 1:
        return one(sys.argv[1])
    for case in CASES:
        r = subprocess.run([sys.executable, __file__, case], capture_output=True, text=True,
                           timeout=150, env=dict(os.environ, DPPO_PEER_DEBUG="1"))
        res = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
        bufs = [l.split("buffer ")[1] for l in r.stderr.splitlines()
                if l.startswith("dppo peer: exchange buffer")]
        print(res[0] if res else f"RESULT {case}: rc {r.returncode} {r.stderr[-400:]}", flush=True)
        print("   buffers: " + " ; ".join(bufs), flush=True)


if __name__ == "__main__":
    main()
