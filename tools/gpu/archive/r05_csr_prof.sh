#!/bin/bash
# Per-kernel times of the partitioned-bucket resolution at C5 (rocprofv3 kernel trace + stats).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/csrprof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 4 --warmup 1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/csrprof/kernel_stats.csv')))
for r in rows:
    n=r['Name']
    if any(k in n for k in ('csr_','fy_','shard','walk')):
        print(n.split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')
PY
