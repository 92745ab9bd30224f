#!/bin/bash
# Round 6 rocprofv3 evidence of the final tree: kernel stats + 4 PMC passes per BASELINE config
# (bench.py), GAE alone at N = 8192 / 65,536.  Summaries: tools/prof_summary.py -> profiles/r06_*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PROF_OUT=$GRAFT_REPO_ROOT/gpurun_out/prof6
CONFIGS="lunar8192 cartpole4096 cheetah4096 c5" GAES="8192|65536 --sets 3" bash profiles/run_profiles_r03.sh || exit 1
