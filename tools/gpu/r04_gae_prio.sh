#!/bin/bash
# Exact GAE at N = 8192: scan-wave priority raised at once (psleep 1) or after the first chunk
# (psleep 5), rocprof A/B, then both timelines (trace build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gpr; mkdir -p $O
DPPO_GAE_PSLEEP=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae_bitexact or gae_vs_oracle or gae_full_size" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name N env
  local sets=16; [ $2 = 65536 ] && sets=3
  env $3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 tools/gae_bench.py --N $2 --sets $sets > $O/b_$1_$2.txt 2>&1 || exit 1
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_' in x['Name']][0]; print('$1 N=$2:', r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
}
for rep in 1 2 3; do
  run ps1_$rep 8192 DPPO_GAE_PSLEEP=1
  run ps5_$rep 8192 DPPO_GAE_PSLEEP=5
done
for rep in 1 2; do
  run ps1_$rep 65536 DPPO_GAE_PSLEEP=1
  run ps5_$rep 65536 DPPO_GAE_PSLEEP=5
done
for P in 1 5; do
  DPPO_GAE_PSLEEP=$P DPPO_LIB=diamond-ppo_amd/build/libdppo_gtrace.so timeout -k 10 120 python tools/gae_trace.py > $O/trace_ps$P.txt 2>&1 || exit 1
  echo "== psleep $P"; grep -v amdgpu.ids $O/trace_ps$P.txt | head -11
done
