#!/bin/bash
# Round 6: GAE load-policy variants (DPPO_GAE_NT 0 / 1 / 5 / 8 / 12): GAE parity per variant, then
# rocprofv3 kernel durations on cold rotating buffers (N = 8192, 16 sets) and the GAE / pack /
# learn events inside C3 learns, 2 interleaved reps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06gae; mkdir -p $O
for V in 1 5 8 12; do
  DPPO_GAE_NT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "gae" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest$V.log 2>&1
  rc=$?; echo "NT=$V parity: $(tail -1 $O/pytest$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do for V in 0 1 5 8 12; do
  DPPO_GAE_NT=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g_${V}_$rep -o run -- python3 tools/gae_bench.py --N 8192 --sets 16 > $O/gb_${V}_$rep.txt 2>&1 || exit 1
  f=$(find $O/g_${V}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]
print('cold NT=$V rep$rep: gae avg %.2f us min %.2f' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3))"
  DPPO_GAE_NT=$V timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 10 --warmup 2 > $O/l_${V}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/l_${V}_$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('learn NT=$V rep$rep', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'gae', k['gae']['us_avg'], 'pack', k['pack']['us_avg'], 'grad', k['grad']['us_avg'])"
done; done
