# The parallel draw into a NumPy array against page-locked memory (what the learner's upload
# slots are), 12 threads.
set -o pipefail
O=gpurun_out/pout; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python tools/perm_par_bench.py --threads 12 --reps 3 --chain 6 > $O/np.$r.log 2>&1 || { tail -3 $O/np.$r.log; exit 1; }
  tail -1 $O/np.$r.log | cut -c1-420
  timeout -k 10 300 python tools/perm_par_bench.py --threads 12 --reps 3 --chain 6 --pinned > $O/pin.$r.log 2>&1 || { tail -3 $O/pin.$r.log; exit 1; }
  tail -1 $O/pin.$r.log | cut -c1-420
done
