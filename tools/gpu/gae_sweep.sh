# GAE N=8192 launch time under the A/B overrides (tile width, workgroups per CU, store type)
for cfg in "A=0" "DPPO_GAE_E=16" "DPPO_GAE_E=16 DPPO_GAE_WGS_PER_CU=2" "DPPO_GAE_WT=1" "A=0"; do
  echo "$cfg: $(env $cfg timeout -k 10 60 python tools/gae_bench.py 2>/dev/null | tail -1)"
done
