#!/bin/bash
# Critic layer's first weight block (and its biases) read before the head rows: parity, bench A/B
# against build/libdppo_latew0.so (the previous order) on C3 / C2 / C4, and the C3 phase trace.
set -o pipefail
O=gpurun_out/w0c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for C in lunar8192 cartpole4096 cheetah4096; do
  for r in 1 2 3; do
    for L in latew0 main; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], d['roofline']['frac'])"
    done
  done
done
PHASE_CONFIG=lunar8192 DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=5000 timeout -k 10 200 python tools/mbw_trace.py > $O/trace.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/trace.txt | head -13
