# The GAE against the new (fastest-pattern) streaming probe, rocprofv3 averages + bench-style events.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/probenew; mkdir -p $O
for rep in 1 2; do for N in 8192 65536; do
  sets=16; [ $N = 65536 ] && sets=3
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g_${N}_$rep -o run -- python3 tools/gae_bench.py --N $N --sets $sets --with-probe > $O/gb_${N}_$rep.txt 2>&1 || exit 1
  f=$(find $O/g_${N}_$rep -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,json
rows=list(csv.DictReader(open('$f')))
g=[x for x in rows if 'gae_pipe' in x['Name']][0]; p=[x for x in rows if 'stream_probe' in x['Name']][0]
b=[json.loads(l) for l in open('$O/gb_${N}_$rep.txt') if l.startswith('{')][-1]
print('N=$N rep$rep: gae avg %.2f us | probe avg %.2f min %.2f us | frac_of_ceiling (events) %.3f' % (float(g['AverageNs'])/1e3, float(p['AverageNs'])/1e3, float(p['MinNs'])/1e3, b['frac_of_ceiling']))"
done; done
