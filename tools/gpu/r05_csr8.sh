#!/bin/bash
# (historical: DPPO_PERM_CSR2, the two-level scatter it measured, is not kept in shuffle.hip)
# Two-level scatter (DPPO_PERM_CSR2=1, opt-in): resolution / learn / global-list tests under it
# (both walk modes), C5 A/B against the one-level scatter, the resolution microbench split, and
# the world-8 member lists.
set -o pipefail
O=gpurun_out/csr8; mkdir -p $O
for W in 0 1; do
DPPO_PERM_CSR2=1 DPPO_PERM_WALK=$W timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dataparallel.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fisher_yates or resolution or swap_targets or c5_full_size or global or cartpole_decay or cheetah_small" > $O/pytest_w$W.log 2>&1
rc=$?; echo "walk=$W: $(tail -1 $O/pytest_w$W.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do for M in 1 0; do
  DPPO_PERM_CSR2=$M timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 > $O/c5.$M.$r.json 2>$O/c5.$M.$r.err || { tail -5 $O/c5.$M.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c5.$M.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('c5 csr2=$M rep$r', round(d['value']/1e6,2), d['ms_per_step'], {c: round(v['ms_total']/v['launches'],3) for c, v in k.items() if c in ('perm','grad','eval')})"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DPPO_PERM_CSR2=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/csr_bench.py --reps 10 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep ms_per_call $O/prof.log
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'csr_' in n or 'fy_' in n: print(n.split('(anonymous namespace)::')[-1].split('(')[0][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
DPPO_PERM_CSR2=1 timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0, 'tools'); import gmb_cap as g
print('two-level: global lists ms', {w: round(g.global_lists_ms(w), 3) for w in (2, 4, 8)})
" 2>&1 | grep -v amdgpu.ids
