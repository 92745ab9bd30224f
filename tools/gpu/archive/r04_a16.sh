#!/bin/bash
# 9-16 actions (untested on the GPU before round 4's end): minibatch gradients against the float64
# oracle and the eval next-value reuse at 10-16 heads.
set -o pipefail
O=gpurun_out/a16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shapes.py tests/test_gpu_eval_reuse.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "head_paths or reuse" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc
