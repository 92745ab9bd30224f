#!/bin/bash
# Kernel split of one rank's global-minibatch member lists at world 8 (configs[4] sizes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/listsprof; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 -c "
import sys; sys.path.insert(0, 'tools'); import gmb_cap as g
print('lists ms world 8', round(g.global_lists_ms(8, reps=10), 3))
" > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
grep "lists ms" $O/run.log
f=$(find $O/p -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/kernel_stats.csv')):
    print(r['Name'].split('(anonymous namespace)::')[-1][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
