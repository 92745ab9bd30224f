# The parallel draw's per-thread rate against the host's load (no GPU use).
set -o pipefail
O=gpurun_out/ddiag; mkdir -p $O
python3 tools/probe/host_load.py
DPPO_PAR_DBG_CHUNKS=1 timeout -k 10 300 python tools/perm_par_bench.py --threads 2,4,8,16 --reps 4 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
python3 tools/probe/host_load.py
tail -1 $O/draw.log
