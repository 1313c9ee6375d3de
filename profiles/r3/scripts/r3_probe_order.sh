#!/bin/bash
# Block order probes on the Zipf image (every block qualifies for the rows
# kernel): control 24, C2's order 33, loads-only 35, loads-only in C2's order 39.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
"$R/tools/box_step.sh" 300 "$O/zipf.log" python3 "$R/tools/bench_c3.py" --variants 24,33,35,39 --rounds 4 --iters 3 || exit 99
grep -h verify_variant "$O/zipf.log" | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("zipf", d["verify_variant"], d["ms_verify_only"])' | tee "$O/summary.txt"
