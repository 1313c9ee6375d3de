set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4b; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 "$O/pytest.log" python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread
grep -q " passed" "$O/pytest.log" && ! grep -q "failed" "$O/pytest.log" || { echo TESTS_FAILED; tail -30 $O/pytest.log; exit 1; }
step 300 "$O/c3_trace.log" rocprofv3 --kernel-trace --stats -d "$O/c3_trace" -o c3 -f csv -- \
    python3 "$R/tools/bench_c3.py" --variants 0 --iters 3 --keep-tail
bash "$R/tools/ab_c3_tail.sh" s4b build/ab/lib_head.so build/ab/lib_new.so 3
step 300 "$O/bench.log" python3 "$R/bench.py"
