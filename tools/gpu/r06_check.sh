#!/bin/bash
# Round 6: the peer fused-step test in its original (uncached-first) order with the detailed
# device error word, the shared-draw test at millisecond draws, then the whole GPU suite and the
# default bench line.
set -o pipefail
mkdir -p gpurun_out/r06
export DPPO_PEER_DEBUG=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 200 --timeout-method thread \
  -k "fused_step or shared_draw" > gpurun_out/r06/peer.log 2>&1 || { echo "peer tests failed"; tail -60 gpurun_out/r06/peer.log; exit 1; }
unset DPPO_PEER_DEBUG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r06/gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06/gpu.log; exit 1; }
tail -3 gpurun_out/r06/gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r06/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r06/bench.log; exit 1; }
tail -1 gpurun_out/r06/bench.log
