#!/bin/bash
# Store-placement probes: C3 rows kernel control 24, deferred result stores 55,
# no result stores 54 (timing only); C2 production 0 vs the per-row scheduling
# barrier 23 (and the streaming ceiling 100) on 1M blocks.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 300 "$O/zipf.log" python3 "$R/tools/bench_c3.py" --variants 24,54,56,57,58 --rounds 3 --iters 3 || exit 99
grep -h verify_variant "$O/zipf.log" | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("zipf", d["verify_variant"], d["ms_verify_only"], d["matches_production"])' | tee "$O/summary.txt"
