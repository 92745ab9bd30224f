#!/bin/bash
# Partitioned buckets, second pass (fused fill + index for the handle's resolution): correctness
# (device resolution public API + learns with device shuffle + global lists), C5 against the
# linked lists, the resolution microbench with the scatter ablations, and the C5 kernel split.
set -o pipefail
O=gpurun_out/csr3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dataparallel.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fisher_yates or swap_targets or c5_full_size or lookahead or cartpole_decay or cheetah_small or deterministic" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for M in 1 0; do
  DPPO_PERM_CSR=$M timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 8 > $O/c5.$M.$r.json 2>$O/c5.$M.$r.err || { tail -5 $O/c5.$M.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c5.$M.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('c5 csr=$M rep$r', round(d['value']/1e6,2), d['ms_per_step'], {c: round(v['ms_total']/v['launches'],3) for c, v in k.items() if c in ('perm','grad','eval')})"
done; done
XARGS="" bash -c true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 4 --warmup 1 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1); cp $f $O/c5_kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/c5_kernel_stats.csv')):
    n=r['Name']
    if 'csr_' in n or 'fy_' in n: print('c5 learn', n.split('(anonymous namespace)::')[-1].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
