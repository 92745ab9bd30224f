#!/bin/bash
# Owner-stagger sweep of the exact GAE kernel (DPPO_GAE_STAGGER cycles between owners' first
# loads): rocprofv3 kernel durations at N = 8192 (16 rotating sets) and 65,536 (3 sets).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gst
STS=${STS:-"640 320 160 0 960"}
NS=${NS:-"8192 65536"}
for rep in 1 2; do
  for st in $STS; do
    for n in $NS; do
      sets=16; [ $n = 65536 ] && sets=3
      DPPO_GAE_STAGGER=$st timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gst/p_${st}_${n}_$rep -o run -- python3 tools/gae_bench.py --N $n --sets $sets > gpurun_out/gst/b_${st}_${n}_$rep.txt 2>&1 || exit 1
      f=$(find gpurun_out/gst/p_${st}_${n}_$rep -name "*kernel_stats.csv" | head -1)
      python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_pipe' in x['Name']][0]; print('stagger $st N=$n rep$rep:', 'avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
    done
  done
done
