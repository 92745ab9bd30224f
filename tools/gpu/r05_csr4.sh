#!/bin/bash
# (historical: the DPPO_ABL_CSR_* timing-only scatter variants it builds against lived in the
# intermediate tree of that measurement, profiles/r05_perm_csr.txt, and are not kept in shuffle.hip)
# Scatter store shape (timing-only, tools/csr_bench.py): step ids only, and one packed 8-B store,
# against the shipped two-array scatter.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/csr4; mkdir -p $O
for nm in main pidonly pack8; do
  lib=diamond-ppo_amd/diamond/libdppo.so; [ $nm != main ] && lib=diamond-ppo_amd/ab/libdppo_csr$nm.so
  DPPO_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$nm -o run -- python3 tools/csr_bench.py --no-check --reps 10 > $O/prof_$nm.log 2>&1 || { tail -5 $O/prof_$nm.log; exit 1; }
  f=$(find $O/p_$nm -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'csr_scatter' in n: print('$nm', n.split('(anonymous namespace)::')[-1].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
