#!/bin/bash
# Old-policy eval change: reuse/eval parity tests on the in-tree library, then the bench A/B
# (tools/gpu/mbw_ab.sh prints the eval column) against build/libdppo_base.so.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval_reuse.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/eval_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/eval_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/mbw_ab.sh ${1:-2} "${2:-cartpole4096 cheetah4096}"
