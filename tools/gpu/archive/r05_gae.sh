# GAE: bit-exact GPU tests with the LDS row swizzle, then swizzle vs no swizzle (ab/libdppo_noswz.so)
# under rocprofv3 at N = 8192 and 65,536 with the streaming ceiling probe beside, and the LDS
# bank-conflict counters of both builds at N = 65,536.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05gae; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "gae" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head; exit $rc; }
lib() { [ "$1" = swz ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for rep in 1 2; do for L in swz noswz; do for N in 8192 65536; do
  sets=16; [ $N = 65536 ] && sets=3
  DPPO_LIB=$(lib $L) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${L}_${N}_$rep -o run -- python3 tools/gae_bench.py --N $N --sets $sets --with-probe > $O/b_${L}_${N}_$rep.txt 2>&1 || exit 1
  f=$(find $O/p_${L}_${N}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,json
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]; p=[x for x in rows if 'stream_probe' in x['Name']][0]
b=json.loads(open('$O/b_${L}_${N}_$rep.txt').read().strip().splitlines()[-1])
print('$L N=$N rep$rep: gae avg %.2f min %.2f us | probe avg %.2f min %.2f us | events gae %.2f probe %.2f frac_of_ceiling %.3f' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3, float(p['AverageNs'])/1e3, float(p['MinNs'])/1e3, b['us_kernel_events'], b['us_probe_kernel_events'], b['frac_of_ceiling']))"
done; done; done
for L in swz noswz; do
  DPPO_LIB=$(lib $L) timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$L -o run -- python3 tools/gae_bench.py --N 65536 --sets 3 --reps 2 > /dev/null 2>&1 || exit 1
  f=$(find $O/pmc_$L -name "*counter_collection.csv" | head -1)
  python3 -c "
import csv,collections
d=collections.defaultdict(float)
for r in csv.DictReader(open('$f')):
  if 'gae_pipe' in r['Kernel_Name']: d[r['Counter_Name']]+=float(r['Counter_Value'])
print('$L N=65536 LDS bank conflict / LDS active = %.1f%%' % (100*d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_LDS_IDX_ACTIVE'],1)))"
done
