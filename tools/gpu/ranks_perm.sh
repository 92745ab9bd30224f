# two concurrent processes drawing permutations: pools spread by LOCAL_RANK vs stacked
for mode in spread stacked; do
  for r in 0 1; do
    if [ $mode = spread ]; then export LOCAL_RANK=$r; else unset LOCAL_RANK; fi
    python tools/perm_thread_bench.py 1048576 > gpurun_out/rp_$mode$r.txt 2>&1 &
  done
  wait
  echo "$mode: $(cat gpurun_out/rp_${mode}0.txt | tail -1) || $(cat gpurun_out/rp_${mode}1.txt | tail -1)"
done
