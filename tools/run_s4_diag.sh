set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4bisect2; mkdir -p $O
export TMPDIR=/tmp
# the round-2 HEAD kernels with only the block-list aux area enlarged (memory layout of the new build)
REVEL_LIB=$R/build/ab/lib_head_bigaux.so timeout -k 10 300 python3 -u -m pytest "$R/tests/test_experiments_gpu.py" "$R/tests/test_gpu.py" -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "not zz_dense and not 64_record" > "$O/head_bigaux.log" 2>&1
echo "rc=$?" >> "$O/head_bigaux.log"
