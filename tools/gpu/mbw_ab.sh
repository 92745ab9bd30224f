#!/bin/bash
# Minibatch-kernel change: production parity suite on the in-tree library, then bench A/B of the
# in-tree library (main) against build/libdppo_base.so on the C2 / C3 / C4 workloads.
#   bash tools/gpu/mbw_ab.sh [reps] [configs]
set -o pipefail
REPS=${1:-2}; CFGS=${2:-"cartpole4096 lunar8192 cheetah4096"}
R=$(pwd)
mkdir -p gpurun_out/mbw_ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/mbw_ab/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/mbw_ab/pytest.log; [ $rc -eq 0 ] || exit $rc
libpath() { [ "$1" = main ] && echo "$R/diamond-ppo_amd/diamond/libdppo.so" || echo "$R/diamond-ppo_amd/build/libdppo_$1.so"; }
for r in $(seq $REPS); do
  for C in $CFGS; do
    for L in main base; do
      DPPO_LIB=$(libpath $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > gpurun_out/mbw_ab/${C}_$L.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('gpurun_out/mbw_ab/${C}_$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,1), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'frac', d['roofline']['frac'], 'eval', k['eval']['us_avg'], 'gae', k['gae']['us_avg'])"
    done
  done
done
