#!/bin/bash
# Full GPU validation of the tree (round 4): pytest -m gpu, smoke(), default bench line.
# Every GPU step has its own time limit and the steps are chained with && (a failed or killed
# step ends the call).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r04_pytest.log 2>&1 \
  && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 \
  && timeout -k 10 500 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?
tail -3 gpurun_out/r04_pytest.log; grep -E "FAILED|ERROR" gpurun_out/r04_pytest.log | head -20
exit $rc
