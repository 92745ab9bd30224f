#!/bin/bash
# Round 6 final check of the tree: the whole GPU suite, smoke(), and the default bench line
# (what the driver runs at round end), then two more default-config C3 lines.
set -o pipefail
mkdir -p gpurun_out/r06final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  > gpurun_out/r06final/gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06final/gpu.log; exit 1; }
tail -2 gpurun_out/r06final/gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06final/smoke.log; exit 1; }
tail -1 gpurun_out/r06final/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06final/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r06final/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r06final/bench.log').read().strip().splitlines()[-1]);print('default', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'], d['roofline_gae']['frac'], d['roofline_gae']['frac_of_ceiling'], {k:(round(v['value']/1e6,1),v['roofline']['frac']) for k,v in d['configs_extra'].items()}, d['cpu_baseline']['value'], d['speedup_vs_reference_equivalent'])"
for r in 1 2; do
  timeout -k 10 300 python bench.py --config lunar8192 --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > gpurun_out/r06final/c3_$r.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r06final/c3_$r.json').read().strip().splitlines()[-1]);print('c3', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'])"
done
