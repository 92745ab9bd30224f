set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/perm_par_bench.py --reps 6 --threads 4,8,12,16 --out gpurun_out/perm_par_r05b.json > gpurun_out/perm_par_r05b.log 2>&1; echo rc $?; tail -1 gpurun_out/perm_par_r05b.log
for e in DPPO_PAR_DBG_NOREC DPPO_PAR_DBG_NOZONE; do env $e=1 timeout -k 10 200 python tools/perm_par_bench.py --reps 3 --threads 8,16 --out gpurun_out/perm_par_r05b_$e.json > gpurun_out/perm_par_r05b_$e.log 2>&1; echo $e rc $?; done
