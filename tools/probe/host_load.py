#!/usr/bin/env python3
"""How busy is this host?  Load average, and the share of each logical CPU busy over 1 s
(/proc/stat), summarised; plus the SMT sibling layout of this process's CPUs."""
import json
import os
import time


def cpu_times():
    t = {}
    for line in open("/proc/stat"):
        if line.startswith("cpu") and line[3].isdigit():
            f = line.split()
            v = list(map(int, f[1:]))
            t[int(f[0][3:])] = (sum(v), v[3] + v[4])
    return t


a = cpu_times()
time.sleep(1.0)
b = cpu_times()
busy = {c: 1.0 - (b[c][1] - a[c][1]) / max(b[c][0] - a[c][0], 1) for c in a}
vals = sorted(busy.values())
sib = {}
for c in sorted(os.sched_getaffinity(0))[:4]:
    try:
        sib[c] = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
    except OSError:
        pass
print(json.dumps({"loadavg": open("/proc/loadavg").read().split()[:3], "cpus": len(vals),
                  "busy_over_50pct": sum(v > 0.5 for v in vals),
                  "busy_mean": round(sum(vals) / len(vals), 3), "siblings": sib}))
