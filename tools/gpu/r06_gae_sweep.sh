#!/bin/bash
# Round 6: GAE at N = 8192 re-swept on this round's tree -- 16-env tiles (two per CU, the second
# tile's loads under the first's scan) against 32-env tiles, and the owners' start stagger
# (0 / 320 / 640 / 960 cycles); rocprofv3 kernel durations on cold rotating buffers, 2 reps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06gs; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 tools/gae_bench.py --N 8192 --sets 16 > $O/$tag.txt 2>&1 || return 1
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]
print('$tag: gae avg %.2f us min %.2f (%s)' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3, g['Name'][:40]))"
}
for rep in 1 2; do
  run e32_$rep DPPO_GAE_E=32 || exit 1
  run e16_$rep DPPO_GAE_E=16 || exit 1
  for st in 0 320 960; do run st${st}_$rep DPPO_GAE_STAGGER=$st || exit 1; done
done
