cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5n
for v in phases p_nodet p_nochain; do
  timeout -k 10 240 python -u tools/fused_phases.py --kernel fused2 --lib build/ab/$v.so --shape small > gpurun_out/r5n/$v.log 2>&1 || exit 1
done
tail -n 1 gpurun_out/r5n/*.log
