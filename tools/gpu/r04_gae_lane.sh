#!/bin/bash
# Lane-per-env tolerance-mode GAE: parity (all GAE tests) then rocprofv3 A/B against the
# LDS-turn form (DPPO_GAE_AFF_LDS=1) and the exact kernel at N = 8192 / 65,536.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/glane; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gae or GAE or affine" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name mode N extra-env
  local sets=16; [ $3 = 65536 ] && sets=3
  local aff=""; [ $2 = aff ] && aff=--affine
  env $4 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$3 -o run -- python3 tools/gae_bench.py --N $3 --sets $sets $aff > $O/b_$1_$3.txt 2>&1 || exit 1
  f=$(find $O/p_$1_$3 -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; r=[x for x in csv.DictReader(open('$f')) if 'gae_' in x['Name']][0]; print('$1 N=$3:', r['Name'][25:45], r['Calls'], 'calls avg %.2f us min %.2f' % (float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))"
}
for rep in 1 2; do
  for n in 8192 65536; do
    run lane_$rep aff $n DPPO_X=0
    run ldsturn_$rep aff $n DPPO_GAE_AFF_LDS=1
    run exact_$rep exact $n DPPO_X=0
  done
done
