#!/bin/bash
# Round 6 batch 5: the exchange-buffer pool against the round-5 free-at-destroy path (diagnosis),
# then the peer tests (fused-step variants in their original order, one process each; the
# second-memory-type refusal) and the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u tools/gpu/r06_coarse_diag.py 2>&1 | tee gpurun_out/r06/coarse_diag5.log || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_peer.py -v --timeout 280 --timeout-method thread \
  -k "fused_step or second_memory_type" > gpurun_out/r06/peer5.log 2>&1 || { echo "peer tests failed"; tail -80 gpurun_out/r06/peer5.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r06/peer5.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  > gpurun_out/r06/gpu5.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06/gpu5.log; exit 1; }
tail -2 gpurun_out/r06/gpu5.log
