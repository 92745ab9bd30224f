# Round 5, batch 3: the full GPU suite + smoke + default bench line on the current tree, then the
# parallel draw with the 64-word accept groups (threads 12 / 16, 2 chunks per thread).
set -o pipefail
bash tools/gpu/full_check.sh || exit 1
grep -q "passed" gpurun_out/full_pytest.log && ! grep -qE "[0-9]+ (failed|error)" gpurun_out/full_pytest.log || exit 1
O=gpurun_out/r05b3; mkdir -p $O
timeout -k 10 300 python tools/perm_par_bench.py --threads 8,12,16 --reps 6 --out $O/draw.json > $O/draw.log 2>&1 || { tail -5 $O/draw.log; exit 1; }
tail -1 $O/draw.log
