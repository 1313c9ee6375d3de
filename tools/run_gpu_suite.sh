set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4fin; mkdir -p $O
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest "$R/tests" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
echo "rc=$?" >> "$O/pytest.log"
