#!/bin/bash
# Tolerance-mode GAE: per-chunk flag hand-off (shipped) vs the round-3 barrier form
# (build/libdppo_affbar.so), rocprofv3 kernel durations at N = 8192 / 65,536, plus the exact
# kernel beside them; GAE parity tests of the shipped library first; then the flag kernel's
# hand-off timeline (build/libdppo_gtrace.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gaff; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae or GAE or affine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name lib mode N stagger
  local sets=16; [ $4 = 65536 ] && sets=3
  local aff=""; [ $3 = aff ] && aff=--affine
  DPPO_GAE_STAGGER=$5 DPPO_LIB=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$4 -o run -- python3 tools/gae_bench.py --N $4 --sets $sets $aff > $O/b_$1_$4.txt 2>&1 || exit 1
  f=$(find $O/p_$1_$4 -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_' in x['Name']][0]; print('$1 N=$4:', r['Name'][:40], r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
}
L=diamond-ppo_amd/diamond/libdppo.so; B=diamond-ppo_amd/build/libdppo_affbar.so
for rep in 1 2; do
  for n in 8192 65536; do
    run flag640_$rep $L aff $n 640
    run flag0_$rep $L aff $n 0
    run bar0_$rep $B aff $n 0
    run exact_$rep $L exact $n 640
  done
done
DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py --affine > $O/trace.txt 2>&1 || exit 1
head -24 $O/trace.txt
