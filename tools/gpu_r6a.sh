set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r6a/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_experiments_gpu.py -m experiment -x -q --timeout 240 --timeout-method thread > gpurun_out/r6a/exp_tests.log 2>&1 || { echo EXP_TESTS_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r6a/bench.json 2> gpurun_out/r6a/bench.err || { echo BENCH_FAILED; exit 1; }
echo ALL_OK
