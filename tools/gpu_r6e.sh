# Round 6: GPU suites on the staged count walk, then an alternating A/B of the
# bench c3 legs, previous product build (build/ab/ctl.so) vs the in-tree one.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_experiments_gpu.py -m experiment -x -q --timeout 240 --timeout-method thread > $O/exp_tests.log 2>&1 || { echo EXP_TESTS_FAILED; exit 1; }
for i in 1 2; do
  for L in build/ab/ctl.so revel_amd/librevel_wal.so; do
    for sh in zipf small; do
      timeout -k 10 200 python -u tools/bench_c3dev.py --lib $L --shape $sh >> $O/ab_c3.log 2>&1 || { echo AB_FAILED; exit 1; }
    done
  done
done
echo ALL_OK
