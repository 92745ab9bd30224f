#!/bin/bash
# Pack kernel 16-B moves for observation widths not a multiple of 4 (and continuous actions):
# parity on the shapes that take that path, then C4 bench A/B against build/libdppo_pre.so.
set -o pipefail
O=gpurun_out/pack2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py tests/test_gpu_eval_reuse.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for r in 1 2; do
  for L in pre main; do
    DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config cheetah4096 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/c4.$L.$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c4.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('cheetah4096 $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'pack', k['pack']['us_avg'], 'eval', k['eval']['us_avg'], 'grad', k['grad']['us_avg'])"
  done
done
