#!/bin/bash
# Round 6 A/B: minibatch + eval kernels compiled with -amdgpu-sched-strategy=max-ilp
# (tools/ab_sched_build.sh -> diamond-ppo_amd/ab_r06/libdppo_maxilp.so) against the default library,
# interleaved pairs at C3, then C4 and C2
set -o pipefail
O=gpurun_out/r06sched; mkdir -p $O
for cfg in lunar8192 lunar8192 lunar8192 cheetah4096 cartpole4096; do for V in def ilp; do
  if [ $V = ilp ]; then export DPPO_LIB=$GRAFT_REPO_ROOT/diamond-ppo_amd/ab_r06/libdppo_maxilp.so; else unset DPPO_LIB; fi
  timeout -k 10 300 python bench.py --config $cfg --no-extra --no-cpu-baseline --no-gae-roofline --steps 20 --warmup 5 > $O/${cfg}_${V}.json 2>$O/${cfg}_${V}.err || { echo "bench $cfg $V failed"; tail -5 $O/${cfg}_${V}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${cfg}_${V}.json').read().strip().splitlines()[-1]);k=d.get('kernels',{});print('$cfg $V', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac'], d['roofline']['us_per_launch'], 'eval', k.get('eval',{}).get('us_avg'))"
done; done
