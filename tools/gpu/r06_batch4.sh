#!/bin/bash
# Round 6 batch 4: the exchange-buffer diagnosis (kept-alive, no-IPC, more uncached, other size),
# then the GPU suite (the coarse / fine fused-step variants aside) and the default bench line.
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u tools/gpu/r06_coarse_diag.py 2>&1 | tee gpurun_out/r06/coarse_diag4.log || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "not (fused_step and (coarse or fine))" > gpurun_out/r06/gpu4.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r06/gpu4.log; exit 1; }
tail -2 gpurun_out/r06/gpu4.log
timeout -k 10 300 python -u bench.py > gpurun_out/r06/bench4.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r06/bench4.log; exit 1; }
tail -1 gpurun_out/r06/bench4.log
