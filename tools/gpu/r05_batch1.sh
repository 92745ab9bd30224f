# Round 5, batch 1: the full GPU suite on the current tree, then the GAE swizzle / ceiling A/B and
# the device-resolution A/B (value walk, epoch-wise) with the global-minibatch scaling cap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -30; exit $rc; }
# GAE: swizzle vs none, with the streaming ceiling beside (rocprofv3 + kernel events)
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for rep in 1 2; do for L in main noswz; do for N in 8192 65536; do
  sets=16; [ $N = 65536 ] && sets=3
  DPPO_LIB=$(lib $L) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g_${L}_${N}_$rep -o run -- python3 tools/gae_bench.py --N $N --sets $sets --with-probe > $O/gb_${L}_${N}_$rep.txt 2>&1 || exit 1
  f=$(find $O/g_${L}_${N}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,json
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]; p=[x for x in rows if 'stream_probe' in x['Name']][0]
b=json.loads(open('$O/gb_${L}_${N}_$rep.txt').read().strip().splitlines()[-1])
print('GAE $L N=$N rep$rep: gae avg %.2f min %.2f us | probe avg %.2f min %.2f | events gae %.2f probe %.2f frac_of_ceiling %.3f' % (float(g['AverageNs'])/1e3, float(g['MinNs'])/1e3, float(p['AverageNs'])/1e3, float(p['MinNs'])/1e3, b['us_kernel_events'], b['us_probe_kernel_events'], b['frac_of_ceiling']))"
done; done; done
for L in main noswz; do
  DPPO_LIB=$(lib $L) timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$L -o run -- python3 tools/gae_bench.py --N 65536 --sets 3 --reps 2 > /dev/null 2>&1 || exit 1
  f=$(find $O/pmc_$L -name "*counter_collection.csv" | head -1)
  python3 -c "
import csv,collections
d=collections.defaultdict(float)
for r in csv.DictReader(open('$f')):
  if 'gae_pipe' in r['Kernel_Name']: d[r['Counter_Name']]+=float(r['Counter_Value'])
print('GAE $L N=65536 LDS bank conflict / LDS active = %.1f%%' % (100*d['SQ_LDS_BANK_CONFLICT']/max(d['SQ_LDS_IDX_ACTIVE'],1)))"
done
# device resolution at C5 one GPU: value walk (default) vs links+solve, each all-epochs / epoch-wise
for rep in 1 2; do for cfg in "1 0" "0 0" "1 1" "0 1"; do set -- $cfg
  DPPO_PERM_WALK=$1 DPPO_PERM_EPOCHWISE=$2 timeout -k 10 300 python bench.py --config c5 --no-extra --no-cpu-baseline --no-gae-roofline --steps 6 --warmup 2 > $O/c5_w$1e$2.$rep.json 2> $O/c5_w$1e$2.$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/c5_w$1e$2.$rep.json').read().strip().splitlines()[-1]);k=d['kernels'];print('C5 walk=$1 epochwise=$2 rep$rep', round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms dev', d['device_ms_per_step'], 'perm', k['perm']['us_avg'], 'us draw', d['host_ms_per_step']['draw'])"
done; done
timeout -k 10 400 python tools/gmb_cap.py --out $O/gmb_cap.json > $O/gmb_cap.log 2>&1; echo gmb rc $?; tail -1 $O/gmb_cap.log | cut -c1-2500
