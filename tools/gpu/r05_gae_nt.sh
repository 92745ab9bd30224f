# GAE owners' streaming variants (DPPO_GAE_NT 0 / 3 / 4 / 7): bit-exact parity per variant, then
# rocprofv3 kernel durations at N = 8192 (16 sets) and 65,536 (3 sets), 2 reps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gaent; mkdir -p $O
for V in 3 4 7; do
  DPPO_GAE_NT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "gae" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest$V.log 2>&1
  rc=$?; echo "NT=$V parity: $(tail -1 $O/pytest$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do for V in 0 3 4 7; do for N in 8192 65536; do
  sets=16; [ $N = 65536 ] && sets=3
  DPPO_GAE_NT=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g_${V}_${N}_$rep -o run -- python3 tools/gae_bench.py --N $N --sets $sets > $O/gb_${V}_${N}_$rep.txt 2>&1 || exit 1
  f=$(find $O/g_${V}_${N}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]
print('NT=$V N=$N rep$rep: gae avg %.2f us min %.2f (%s)' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3, g['Name'][:60]))"
done; done; done
