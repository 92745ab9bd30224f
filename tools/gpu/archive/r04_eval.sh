#!/bin/bash
# Old-policy eval kernel: compile-time LDS layout + 16-B observation loads.  Parity of the eval /
# act paths, then bench A/B against build/libdppo_pre.so on C3 / C2 / C4.
set -o pipefail
O=gpurun_out/ev; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_eval_reuse.py tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_rollout_ckpt.py tests/test_gpu_shapes.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for C in lunar8192 cartpole4096 cheetah4096; do
  for r in 1 2; do
    for L in pre main; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'eval', k['eval']['us_avg'], 'grad', k['grad']['us_avg'])"
    done
  done
done
