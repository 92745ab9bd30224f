#!/bin/bash
# Exact GAE at N = 8192: the scan wave's poll back-off (DPPO_GAE_PSLEEP 0 / 1 / 2) and 64-env
# tiles on 128 workgroups (DPPO_GAE_E=64), rocprofv3 A/B; parity of the exact kernel first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gps; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae or GAE" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
DPPO_GAE_PSLEEP=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae_bitexact or gae_vs_oracle or gae_full_size" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -1 $O/pytest.log; tail -1 $O/pytest2.log
run() {  # name N env
  local sets=16; [ $2 = 65536 ] && sets=3
  env $3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 tools/gae_bench.py --N $2 --sets $sets > $O/b_$1_$2.txt 2>&1 || exit 1
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_' in x['Name']][0]; print('$1 N=$2:', r['Name'][25:50], r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
}
for rep in 1 2 3; do
  run ps0_$rep 8192 DPPO_GAE_PSLEEP=0
  run ps1_$rep 8192 DPPO_GAE_PSLEEP=1
  run ps2_$rep 8192 DPPO_GAE_PSLEEP=2
  run e64_$rep 8192 DPPO_GAE_E=64
done
for rep in 1 2; do
  run ps0_$rep 65536 DPPO_GAE_PSLEEP=0
  run ps2_$rep 65536 DPPO_GAE_PSLEEP=2
done
DPPO_GAE_PSLEEP=2 DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py > $O/trace_ps2.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/trace_ps2.txt | head -12
