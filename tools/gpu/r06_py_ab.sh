#!/bin/bash
# Round 6: C3 learns with the current tree (look-ahead depth 3 and 2) against the batch-4 tree
# (diamond package + library of commit 527bb01, tools/ab_py/r527), 3 interleaved rounds.
set -o pipefail
O=gpurun_out/r06py2; mkdir -p $O
cat /proc/loadavg
for r in 1 2 3; do for V in new3 new2 old; do
  unset DPPO_PY_ROOT DPPO_PERM_DEPTH
  [ $V = old ] && export DPPO_PY_ROOT=$GRAFT_REPO_ROOT/tools/ab_py/r527
  [ $V = new2 ] && export DPPO_PERM_DEPTH=2
  timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/c3_${V}_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/c3_${V}_$r.json').read().strip().splitlines()[-1]);h=d['host_ms_per_step'];print('$V rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'perms', h['perms'], 'draw', h['draw'], 'slot', h['slot_wait'], 'unchained', round(d['value_unchained_obs']/1e6,2))"
done; done
cat /proc/loadavg
