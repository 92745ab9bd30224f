#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u tools/gpu/r06_coarse_diag.py 2>&1 | tee gpurun_out/r06/coarse_diag2.log && \
bash tools/gpu/r06_gae_nt.sh 2>&1 | tee gpurun_out/r06/gae_nt.log && \
bash tools/gpu/r06_recpad.sh 2>&1 | tee gpurun_out/r06/recpad.log
