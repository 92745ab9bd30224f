#!/bin/bash
# Round 6: bench.py --gpus 8 rehearsed on the one-GPU box (8 ranks share GPU 0, gloo group, peer
# exchange; the global-minibatch legs run the node-shared draw with seven followers holding slots)
set -o pipefail
mkdir -p gpurun_out/r06reh
DPPO_BENCH_REHEARSE=1 MASTER_ADDR=127.0.0.1 timeout -k 10 600 python -u bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r06reh/bench8.log 2>&1 || { echo "rehearsal failed"; tail -40 gpurun_out/r06reh/bench8.log; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r06reh/bench8.log').read().strip().splitlines()[-1])
mg=d['multi_gpu'];print('n_gpus',d['n_gpus'],'value',round(d['value']/1e6,2),'exchange',mg['exchange']['transport'],mg['exchange']['peer_selftest'],mg['exchange']['memory'])
print({k:(v.get('update_steps_per_s'), v.get('minibatches')) for k,v in mg.items() if k.startswith('c5_strong')}, mg.get('c5_update_steps_speedup_vs_world1'))
print('share', mg['c5_strong_global'].get('perm_share'))"
