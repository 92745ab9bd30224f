#!/bin/bash
# Gaussian-head (C4) minibatch kernel after keeping its phase-8/9 math scalar: parity of the
# continuous paths, C4 bench A/B against build/libdppo_pre.so, then the C3 / C2 phase traces.
set -o pipefail
O=gpurun_out/c4pk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -q -x -k "cont or cheetah or C4 or Gaussian or pendulum or learn_trace" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for r in 1 2 3; do
  for L in pre main; do
    DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config cheetah4096 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/c4.$L.$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c4.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('cheetah4096 $L', round(d['value']/1e6,2), d['ms_per_step'], 'dev', d['device_ms_per_step'], 'eval', k['eval']['us_avg'], 'grad', k['grad']['us_avg'], d['roofline']['frac'])"
  done
done
for C in lunar8192 cartpole4096; do
  PHASE_CONFIG=$C DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=5000 timeout -k 10 200 python tools/mbw_trace.py > $O/trace_$C.txt 2>&1 || exit 1
  echo "== $C"; grep -v amdgpu.ids $O/trace_$C.txt | head -13
done
