#!/bin/bash
# Round 6: where the host time of a host-bound C3 learn goes on this box -- CPU topology, the
# standalone draft rate (perm_numpy on a thread, C3 size), and a per-learn timeline of the learn loop.
set -o pipefail
O=gpurun_out/r06hd; mkdir -p $O
nproc; cat /proc/loadavg; grep -c processor /proc/cpuinfo
timeout -k 10 120 python tools/perm_thread_bench.py 1048576 2>&1 | tail -3
timeout -k 10 200 python -u tools/host_timeline.py --config lunar8192 --learns 24 > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 1; }
head -3 $O/timeline.txt; tail -2 $O/timeline.txt
