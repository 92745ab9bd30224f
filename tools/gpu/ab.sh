#!/bin/bash
# Generic bench A/B of variant libraries (diamond-ppo_amd/ab/libdppo_<name>.so) against the shipped
# one, interleaved, bench events per kernel.
#   bash tools/gpu/ab.sh "<variants>" "<configs>" [reps] [parity-variants]
# parity-variants: variants whose production parity (tests/test_gpu_production.py) runs first
# (timing-only ablations, which compute wrong results, are left out of it); PARITY_TESTS overrides
# the test files.
set -o pipefail
V=$1; CS=${2:-"cartpole4096 lunar8192 cheetah4096"}; REPS=${3:-2}; PAR=${4:-}
O=gpurun_out/ab; mkdir -p $O
for P in $PAR; do
  DPPO_LIB=diamond-ppo_amd/ab/libdppo_$P.so timeout -k 10 900 python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_production.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$P.log 2>&1
  rc=$?; echo "parity $P: $(tail -1 $O/pytest_$P.log)"; [ $rc -eq 0 ] || exit $rc
done
lib() { [ "$1" = main ] && echo diamond-ppo_amd/diamond/libdppo.so || echo diamond-ppo_amd/ab/libdppo_$1.so; }
for r in $(seq 1 $REPS); do for C in $CS; do for L in main $V; do
  st=20; [ $C = c5 ] && st=8
  DPPO_LIB=$(lib $L) timeout -k 10 300 python bench.py --config $C --no-extra --no-cpu-baseline --no-gae-roofline --steps $st > $O/$C.$L.$r.json 2>$O/$C.$L.$r.err || { tail -5 $O/$C.$L.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$C.$L.$r.json').read().strip().splitlines()[-1]);k=d['kernels'];print('$C $L rep$r', round(d['value']/1e6,2), d['ms_per_step'], 'radam', k['reduce_adam']['us_avg'], 'grad', k['grad']['us_avg'], 'frac', d['roofline']['frac'])"
done; done; done
