#!/bin/bash
# A/B of the GAE kernel: the in-tree libdppo.so (new) against build/libdppo_base.so, rocprofv3
# kernel durations at N = 8192 and 65,536, ABAB; GAE parity tests on the new library first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae or GAE" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gab/pytest.log 2>&1 || { tail -20 gpurun_out/gab/pytest.log; exit 1; }
tail -2 gpurun_out/gab/pytest.log
for rep in 1 2; do
  for v in new base; do
    lib=diamond-ppo_amd/diamond/libdppo.so; [ $v = base ] && lib=diamond-ppo_amd/build/libdppo_base.so
    for n in 8192 65536; do
      sets=16; [ $n = 65536 ] && sets=3
      DPPO_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gab/p_${v}_${n}_$rep -o run -- python3 tools/gae_bench.py --N $n --sets $sets > gpurun_out/gab/b_${v}_${n}_$rep.txt 2>&1 || exit 1
      f=$(find gpurun_out/gab/p_${v}_${n}_$rep -name "*kernel_stats.csv" | head -1)
      python3 -c "import csv,sys; r=[x for x in csv.DictReader(open('$f')) if 'gae_pipe' in x['Name']][0]; print('$v N=$n rep$rep:', r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
    done
  done
done
DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py > gpurun_out/gab/trace.txt 2>&1 || exit 1
head -24 gpurun_out/gab/trace.txt
