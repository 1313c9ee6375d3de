set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_count; mkdir -p $O
for i in 1 2; do
  for L in lib_new lib_nostore lib_pipe; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$L.log" python3 "$R/tools/bench_c3.py" --lib "$R/build/ab/$L.so" --variants 0 --rounds 2 --iters 5 || exit 99
  done
done
