#!/bin/bash
# Final tree after the partitioned-bucket resolution: full GPU suite, smoke, default bench line,
# and the C5 kernel stats (rocprofv3).
set -o pipefail
bash tools/gpu/full_check.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/final3; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 > $O/c5_bench.json 2> $O/c5_prof.log || { tail -5 $O/c5_prof.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1); cp $f $O/c5_kernel_stats.csv
python3 -c "import json;d=json.loads(open('$O/c5_bench.json').read().strip().splitlines()[-1]);print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
