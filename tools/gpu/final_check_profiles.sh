#!/bin/bash
# Round-end evidence in one call: full validation (tools/gpu/full_check.sh: pytest -m gpu, smoke,
# default bench line), then the rocprofv3 kernel-stats + PMC passes of every BASELINE config and
# the GAE sizes (profiles/run_profiles_r03.sh).
set -o pipefail
bash tools/gpu/full_check.sh || exit 1
grep -q "passed" gpurun_out/full_pytest.log && ! grep -qE "[0-9]+ failed" gpurun_out/full_pytest.log || exit 1
CONFIGS="cartpole4096 lunar8192 cheetah4096 c5" GAES="8192|65536 --sets 3" bash profiles/run_profiles_r03.sh
