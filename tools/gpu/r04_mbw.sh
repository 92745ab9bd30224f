#!/bin/bash
# Minibatch-kernel A/B (round 4): parity of the shipped library on the shapes the change touches,
# then bench A/B of build/libdppo_r04base.so (before) against the shipped library (after) on C4 /
# C3 / C2, the half-slab timing ablation (build/libdppo_halfslab.so: the upper bound of a pairwise
# slab hand-off), and the C4 phase trace of the new kernel.
set -o pipefail
mkdir -p gpurun_out/r04mbw
O=gpurun_out/r04mbw
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -m gpu -q -k "cheetah or cont or C4 or Gaussian or learn_trace or shapes or 7 or 8" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head; [ $rc -eq 0 ] || exit $rc
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for C in cheetah4096 lunar8192 cartpole4096; do
  for r in 1 2; do
    for L in r04base main; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', d['value'], d['ms_per_step'], 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'radam', k['reduce_adam']['us_avg'], d['roofline']['frac'])"
    done
  done
done
for C in cartpole4096 lunar8192; do
  for L in main halfslab; do
    DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/hs.$C.$L.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/hs.$C.$L.json').read().strip().splitlines()[-1]);k=d['kernels'];print('halfslab-ablation $C $L', d['value'], 'grad', k['grad']['us_avg'], 'radam', k['reduce_adam']['us_avg'])"
  done
done
PHASE_CONFIG=cheetah4096 DPPO_LIB=diamond-ppo_amd/build/libdppo_trace.so WARM_LAUNCHES=20000 timeout -k 10 200 python tools/mbw_trace.py > $O/trace_cheetah4096.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/trace_cheetah4096.txt | head -20
