cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5o
timeout -k 10 480 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r5o/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
for v in phases p_two p_nodet p_nochain; do
  timeout -k 10 240 python -u tools/fused_phases.py --kernel fused2 --lib build/ab/$v.so --shape small > gpurun_out/r5o/$v.log 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/ab_fused.py --hook revel_debug_set_fused --on 2 --rounds 3 > gpurun_out/r5o/ab_fused2.log 2>&1
echo "rc=$?"
for v in phases p_two p_nodet p_nochain; do echo $v; tail -n 1 gpurun_out/r5o/$v.log | cut -c1-260; done
tail -n 1 gpurun_out/r5o/ab_fused2.log
