#!/bin/bash
# Round 6 batch 3: the exchange-buffer diagnosis with the last word read and the acquire-fence
# variant; GAE non-temporal loads (NT=1) against plain, 4 more interleaved reps cold and in-learn.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u tools/gpu/r06_coarse_diag.py 2>&1 | tee gpurun_out/r06/coarse_diag3.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06gae; mkdir -p $O
for rep in 3 4 5 6; do for V in 0 1; do
  DPPO_GAE_NT=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g_${V}_$rep -o run -- python3 tools/gae_bench.py --N 8192 --sets 16 > $O/gb_${V}_$rep.txt 2>&1 || exit 1
  f=$(find $O/g_${V}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]
print('cold NT=$V rep$rep: gae avg %.2f us min %.2f' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3))"
  DPPO_GAE_NT=$V timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --steps 20 --warmup 3 > $O/l_${V}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/l_${V}_$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];g=d['roofline_gae'];print('learn NT=$V rep$rep', round(d['value']/1e6,2), d['ms_per_step'], 'gae', k['gae']['us_avg'], 'pack', k['pack']['us_avg'], 'roofline_gae us', g.get('us_per_launch', g.get('kernel_us')), 'ceiling', g.get('ceiling_us'), 'frac_ceil', g.get('frac_of_ceiling'))"
done; done
