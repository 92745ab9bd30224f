#!/bin/bash
# Round-3 rocprofv3 evidence (run on the GPU box via gpurun):
#  * bench.py per BASELINE config (CONFIGS: cartpole4096 lunar8192 cheetah4096 c5): kernel trace +
#    stats, then four separate --pmc passes (SQ occupancy / stall / MFMA mix, LDS, FETCH_SIZE,
#    WRITE_SIZE) -- counters never combined with tracing domains;
#  * GAE alone (tools/gae_bench.py) at N = 8192 and 65,536, both modes: kernel trace + HBM bytes.
# Output: gpurun_out/prof3/<name>/...; summarise with tools/prof_summary.py.
# CONFIGS / GAES (|-separated, empty = none) select the runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${PROF_OUT:-$R/gpurun_out/prof3}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
CONFIGS=${CONFIGS:-cartpole4096 lunar8192 cheetah4096 c5}
for C in $CONFIGS; do
  D=$OUT/$C
  mkdir -p $D
  B="$R/bench.py --no-cpu-baseline --no-gae-roofline --no-extra --config $C"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- \
    python3 $B --steps 6 --warmup 2 > $D/kt.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    --output-format csv -d $D/pmc1 -o p1 -- python3 $B --steps 2 --warmup 1 > $D/pmc1.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM \
    --output-format csv -d $D/pmc2 -o p2 -- python3 $B --steps 2 --warmup 1 > $D/pmc2.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc3 -o p3 -- \
    python3 $B --steps 2 --warmup 1 > $D/pmc3.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $D/pmc4 \
    -o p4 -- python3 $B --steps 2 --warmup 1 > $D/pmc4.log 2>&1 || exit 1
  echo "$C done"
done
GAES=${GAES-"8192|8192 --affine|65536 --sets 3|65536 --sets 3 --affine"}
IFS='|' read -ra GLIST <<< "$GAES"
for G in "${GLIST[@]}"; do
  set -- $G
  D=$OUT/gae$1$(echo "$G" | grep -q affine && echo _affine)
  mkdir -p $D
  A="$R/tools/gae_bench.py --N $G"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/gkt -o gkt -- \
    python3 $A --reps 4 > $D/gkt.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/gpmc3 -o g3 -- \
    python3 $A --reps 1 > $D/gpmc3.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $D/gpmc4 \
    -o g4 -- python3 $A --reps 1 > $D/gpmc4.log 2>&1 || exit 1
  echo "gae $G done"
done
