#!/bin/bash
# Round 6: the reference-exact mode's per-rank target upload (134 MB per learn at configs[4]):
# H2D rate from pinned and from registered shared memory, world-8 share learns alone / with one
# upload per learn / with uploads back to back (tools/upload_rate.py); then a short kernel +
# memory-copy trace of the same tool (is the upload a DMA-engine copy or a blit kernel?)
set -o pipefail
mkdir -p gpurun_out/r06up
timeout -k 10 400 python -u tools/upload_rate.py --reps 5 --out gpurun_out/r06up/upload.json > gpurun_out/r06up/upload.log 2>&1 || { echo "upload_rate failed"; tail -30 gpurun_out/r06up/upload.log; exit 1; }
tail -1 gpurun_out/r06up/upload.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06up/prof -o up -- python3 $GRAFT_REPO_ROOT/tools/upload_rate.py --reps 1 --steps 8 > $GRAFT_REPO_ROOT/gpurun_out/r06up/prof.log 2>&1 || { echo "profile failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r06up/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r06up/prof -name "*stats*.csv" | head -5
