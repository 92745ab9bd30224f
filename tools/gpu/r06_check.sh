#!/bin/bash
# Round 6: the coarse-buffer diagnosis (tools/gpu/r06_coarse_diag.py), the shared-draw test at
# millisecond draws, then the whole GPU suite and the default bench line.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u tools/gpu/r06_coarse_diag.py > gpurun_out/r06/coarse_diag.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/r06/coarse_diag.log; exit 1; }
cat gpurun_out/r06/coarse_diag.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 200 --timeout-method thread \
  -k "shared_draw" > gpurun_out/r06/share.log 2>&1 || { echo "share test failed"; tail -60 gpurun_out/r06/share.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "not coarse" > gpurun_out/r06/gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06/gpu.log; exit 1; }
tail -3 gpurun_out/r06/gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r06/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r06/bench.log; exit 1; }
tail -1 gpurun_out/r06/bench.log
