# quick bench: default config without extras, then the lunar8192 config
B="python bench.py --no-extra --no-cpu-baseline --no-gae-roofline --steps 30 --warmup 5"
timeout -k 10 200 $B > gpurun_out/q_c2.json 2> gpurun_out/q_c2.err &&
timeout -k 10 200 $B --config lunar8192 > gpurun_out/q_c3.json 2> gpurun_out/q_c3.err
