#!/bin/bash
# Exact GAE at N = 65,536 (64-env tiles): the scan wave's poll back-off (DPPO_GAE_PSLEEP 0 / 1),
# 3 interleaved rocprofv3 reps each, and 32-env tiles (DPPO_GAE_E=32) for reference.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g65; mkdir -p $O
run() {  # name N env
  local sets=16; [ $2 = 65536 ] && sets=3
  env $3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 tools/gae_bench.py --N $2 --sets $sets > $O/b_$1_$2.txt 2>&1 || exit 1
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_' in x['Name']][0]; print('$1 N=$2:', r['Name'][25:50], r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
}
for rep in 1 2 3; do
  run ps0_$rep 65536 DPPO_GAE_PSLEEP=0
  run ps1_$rep 65536 DPPO_GAE_PSLEEP=1
done
run e32_1 65536 DPPO_GAE_E=32
