#!/bin/bash
# 4-head MFMA back-propagation: parity on the shapes that use it, then C3 bench A/B against the
# VALU form (build/libdppo_noda.so), 3 pairs; GAE at 65,536 with the poll back-off.
set -o pipefail
O=gpurun_out/r04da; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for r in 1 2 3; do
  for L in noda main; do
    DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/c3.$L.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c3.$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('C3 $L', d['value'], d['ms_per_step'], 'grad', k['grad']['us_avg'], d['roofline']['frac'])"
  done
done
