#!/bin/bash
# Result-store probes (experiment arms, timing only): control 24, no result
# stores 54, nontemporal 56, results into a private line-aligned 64-slot region
# per block with all lanes (59: whole lines) or lanes < n (60: partial lines).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 300 "$O/zipf.log" python3 "$R/tools/bench_c3.py" --variants ${VARS:-24,54,56,59,60} --rounds ${ROUNDS:-3} --iters 3 || exit 99
grep -h verify_variant "$O/zipf.log" | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("zipf", d["verify_variant"], d["ms_verify_only"])' | tee "$O/summary.txt"
