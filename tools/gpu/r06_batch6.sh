#!/bin/bash
# Round 6 batch 6: the whole GPU suite, smoke, the default bench line, and three more C3 lines
# (host placement of the draws reported in each).
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  > gpurun_out/r06/gpu6.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06/gpu6.log; exit 1; }
tail -2 gpurun_out/r06/gpu6.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke6.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06/smoke6.log; exit 1; }
tail -1 gpurun_out/r06/smoke6.log
timeout -k 10 300 python -u bench.py > gpurun_out/r06/bench6.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r06/bench6.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r06/bench6.log').read().strip().splitlines()[-1]);print('default', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'], d['host_placement'], d['cpu_baseline'].get('reference_equivalent_value'))"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > gpurun_out/r06/c3_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r06/c3_$r.json').read().strip().splitlines()[-1]);print('c3', round(d['value']/1e6,2), d['ms_per_step'], d['host_ms_per_step']['draw'], d['host_placement'])"
done
