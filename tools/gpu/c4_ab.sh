#!/bin/bash
# C4 (HalfCheetah, D=17, A=6) minibatch-kernel A/B: parity of the sample-split path, then the
# cheetah4096 bench with the two-team kernel (0) and the sample-split kernel (1).
set -o pipefail
mkdir -p gpurun_out
DPPO_MBW_CONT6=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py -m gpu -q -k "cheetah or cont or C4" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c4_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c4_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    DPPO_MBW_CONT6=$v timeout -k 10 200 python bench.py --config cheetah4096 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > gpurun_out/c4_ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/c4_ab_$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('CONT6=$v', d['value'], d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], d['roofline']['frac'])"
  done
done
