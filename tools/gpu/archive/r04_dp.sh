#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dataparallel.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r04_dp.log | head -30; exit $rc
