#!/bin/bash
# LLVM machine-scheduler strategy A/B for the minibatch and eval kernels: the shipped default
# (GCN max-occupancy) against max-ilp and max-memory-clause builds of mbwave.hip + mlp.hip
# (build/libdppo_maxilp.so, build/libdppo_maxmemoryclause.so) -- parity on the traces, then bench.
set -o pipefail
O=gpurun_out/sched; mkdir -p $O
for L in maxilp maxmemoryclause; do
  DPPO_LIB=diamond-ppo_amd/build/libdppo_$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "learn_trace or golden" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$L.log 2>&1
  rc=$?; tail -1 $O/pytest_$L.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_$L.log | head -20; exit $rc; }
done
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/build/libdppo_$1.so; }
for C in lunar8192 cartpole4096 cheetah4096; do
  for r in 1 2; do
    for L in main maxilp maxmemoryclause; do
      DPPO_LIB=$(lib $L) timeout -k 10 200 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 > $O/$C.$L.$r.json 2>/dev/null || exit 1
      python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L', round(d['value']/1e6,2), 'dev', d['device_ms_per_step'], 'grad', k['grad']['us_avg'], 'eval', k['eval']['us_avg'])"
    done
  done
done
