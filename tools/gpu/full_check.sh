#!/bin/bash
# Full GPU validation of the tree: pytest -m gpu, smoke(), default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/full_pytest.log; grep -E "FAILED|ERROR" gpurun_out/full_pytest.log | head -20
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/full_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err
echo "bench rc=$?"
python3 -c "import json;d=json.loads(open('gpurun_out/full_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gae']['us_per_launch'], d['roofline_gae_65536']['exact']['frac'], d['cpu_baseline']['value'])"
