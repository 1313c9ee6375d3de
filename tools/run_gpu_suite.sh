set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4scan; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
echo "rc=$?" >> "$O/pytest.log"
