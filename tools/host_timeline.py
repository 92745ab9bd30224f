#!/usr/bin/env python3
"""Per-learn host timeline of bench.py's C3 loop (round 6: some boxes ran the learn host-bound).
Wraps the learner's draft / slot / enqueue steps with time stamps and prints, per learn, the
launching thread's waits and each draft's draw and swap-completion times, plus the CPU topology
this process may use.  Diagnosis only.

    python tools/host_timeline.py [--config lunar8192] [--learns 24]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "diamond-ppo_amd")]


def topology():
    allowed = sorted(os.sched_getaffinity(0))
    doms = {}
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                doms.setdefault(f.read().strip(), []).append(c)
        except OSError:
            doms.setdefault("?", []).append(c)
    with open("/proc/loadavg") as f:
        load = f.read().split()[:3]
    return {"allowed": len(allowed), "l3_domains": {k: len(v) for k, v in doms.items()},
            "loadavg": load, "cpu_count": os.cpu_count()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="lunar8192")
    ap.add_argument("--learns", type=int, default=24)
    a = ap.parse_args()
    import torch
    import bench
    from diamond import engine as E
    from diamond import _native as N
    print("topology", topology(), flush=True)
    import diamond
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model, T, Nc, D, A, cont, pt, ptr, scaling = bench.CONFIGS[a.config]
    Cfg = diamond.ContinuousPPOConfig if cont else diamond.PPOConfig
    Agent = diamond.ContinuousPPO if cont else diamond.PPO
    cfg = Cfg(rollout_steps=T, num_envs=Nc, verbose=False, total_steps=10 ** 12)
    agent = Agent(None, cfg, envs=bench.SpecEnvs(D, A, cont))
    L = agent._learner
    ev = []
    t00 = time.perf_counter()
    stamp = lambda what, **kw: ev.append((time.perf_counter() - t00, threading.current_thread().name, what, kw))  # noqa: E731
    fin, start, pbuf = E.NativeLearner._finish, L._start_draft, L.handle.perm_buffer

    def _finish(d):
        stamp("finish_wait")
        fin(d)
        stamp("finish_done", t_draw=d.get("t_draw"))

    def _start_draft(key, pos):
        stamp("draft_submit")
        return start(key, pos)

    def perm_buffer(slot):
        stamp("slot_wait", slot=slot)
        r = pbuf(slot)
        stamp("slot_done", slot=slot)
        return r

    import gc
    gc.callbacks.append(lambda phase, info: stamp("gc_" + phase, gen=info["generation"]))
    lrn = L.learn

    def learn_w(*args, **kw):
        r = lrn(*args, **kw)
        stamp("learn_done")
        return r

    L.learn = learn_w
    E.NativeLearner._finish = staticmethod(_finish)
    L._start_draft = _start_draft
    L.handle.perm_buffer = perm_buffer
    ro = bench.synth_rollout(T, Nc, D, A, cont, pt, ptr, seed=0, device=dev)[0]
    for _ in range(6):
        agent.learn_device(ro)
    torch.cuda.synchronize()
    ev.clear()
    t0 = time.perf_counter()
    for i in range(a.learns):
        stamp("learn", i=i)
        agent.learn_device(ro)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{a.learns} learns {el * 1e3 / a.learns:.3f} ms each", flush=True)
    for t, th, what, kw in ev:
        print(f"{t * 1e3:9.3f} {th[:14]:14s} {what:13s} {kw}")
    print("host_seconds", {k: round(v, 4) if isinstance(v, float) else v
                            for k, v in L.host_seconds.items()})
    print("placement", N.perm_domain())


if __name__ == "__main__":
    main()
