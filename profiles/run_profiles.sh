#!/bin/bash
# Collects the committed rocprofv3 evidence for bench.py (run on the GPU box via gpurun).
#   kernel trace + stats (timing), then separate PMC passes (SQ occupancy/stall/MFMA mix, HBM
#   FETCH_SIZE, WRITE_SIZE) -- counters never combined with tracing domains.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-gae-roofline --no-extra ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 $B --steps 10 --warmup 2 > $OUT/kt.log 2>&1
echo "kernel trace done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --output-format csv -d $OUT/pmc1 -o p1 -- python3 $B --steps 2 --warmup 1 > $OUT/pmc1.log 2>&1
echo "pmc1 done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM \
  --output-format csv -d $OUT/pmc2 -o p2 -- python3 $B --steps 2 --warmup 1 > $OUT/pmc2.log 2>&1
echo "pmc2 done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o p3 -- \
  python3 $B --steps 2 --warmup 1 > $OUT/pmc3.log 2>&1
echo "pmc3 done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc4 \
  -o p4 -- python3 $B --steps 2 --warmup 1 > $OUT/pmc4.log 2>&1
echo "pmc4 done"
# GAE at N = 8192 (bench.py roofline_gae): 16 rotating 23 MB buffer sets
G="$R/tools/gae_bench.py --N 8192"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gkt -o gkt -- \
  python3 $G --reps 4 > $OUT/gkt.log 2>&1
echo "gae kernel trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/gpmc3 -o g3 -- \
  python3 $G --reps 1 > $OUT/gpmc3.log 2>&1
echo "gae pmc3 done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/gpmc4 \
  -o g4 -- python3 $G --reps 1 > $OUT/gpmc4.log 2>&1
echo "gae pmc4 done"
