#!/bin/bash
# (historical: the DPPO_ABL_CSR_* timing-only scatter variants it builds against lived in the
# intermediate tree of that measurement, profiles/r05_perm_csr.txt, and are not kept in shuffle.hip)
# Partitioned-bucket resolution alone (tools/csr_bench.py, configs[4] size): the default library
# (checked bit-exact, both modes), the linked lists (DPPO_PERM_CSR=0), and the two timing-only
# scatter ablations, each under rocprofv3 for the per-pass split.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/csr2; mkdir -p $O
run() {  # name env...
  local nm=$1; shift
  env "$@" timeout -k 10 200 python3 tools/csr_bench.py $XARGS > $O/$nm.json 2> $O/$nm.err || { tail -5 $O/$nm.err; exit 1; }
  cat $O/$nm.json
}
XARGS="" run csr DPPO_PERM_CSR=1
XARGS="--walk 1" run csr_walk DPPO_PERM_CSR=1
XARGS="" run lists DPPO_PERM_CSR=0
XARGS="--no-check" run nostore DPPO_LIB=diamond-ppo_amd/ab/libdppo_csrnost.so
XARGS="--no-check" run noatomic DPPO_LIB=diamond-ppo_amd/ab/libdppo_csrnoat.so
for nm in csr nost noat; do
  lib=diamond-ppo_amd/diamond/libdppo.so; [ $nm = nost ] && lib=diamond-ppo_amd/ab/libdppo_csrnost.so; [ $nm = noat ] && lib=diamond-ppo_amd/ab/libdppo_csrnoat.so
  chk=""; [ $nm != csr ] && chk="--no-check"
  DPPO_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$nm -o run -- python3 tools/csr_bench.py --no-check --reps 10 > $O/prof_$nm.log 2>&1 || { tail -5 $O/prof_$nm.log; exit 1; }
  f=$(find $O/p_$nm -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'csr_' in n or 'fy_' in n: print('$nm', n.split('(anonymous namespace)::')[-1].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
