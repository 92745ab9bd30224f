# Round 5 rocprofv3 evidence: kernel stats + 4 PMC passes per BASELINE config (bench.py), GAE alone
# at N = 8192 / 65,536, and the reduce_adam timeline (timing-only DPPO_RA_TRACE build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PROF_OUT=$GRAFT_REPO_ROOT/gpurun_out/prof5
CONFIGS="lunar8192 cartpole4096 cheetah4096 c5" GAES="8192|65536 --sets 3" bash profiles/run_profiles_r03.sh || exit 1
for C in lunar8192 cartpole4096; do
  PHASE_CONFIG=$C DPPO_LIB=diamond-ppo_amd/ab/libdppo_ratrace.so timeout -k 10 200 python tools/ra_trace.py > gpurun_out/prof5/ra_trace_$C.txt 2>&1 || { tail -5 gpurun_out/prof5/ra_trace_$C.txt; exit 1; }
  tail -12 gpurun_out/prof5/ra_trace_$C.txt
done
