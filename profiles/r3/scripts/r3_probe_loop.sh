#!/bin/bash
# Row-loop probes (experiment arms, wrong CRCs): loads-only 35 / 39 (sorted /
# C2 order), row loop alone 43 / 44 (sorted / C2 order), 45 (C2 order, 16-row
# ring); C2 and the streaming ceiling on the same 4 GiB.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 300 "$O/zipf.log" python3 "$R/tools/bench_c3.py" --variants 24,55,54 --rounds 4 --iters 3 || exit 99
$S 300 "$O/full.log" python3 "$R/tools/bench_c3.py" --image full --variants 24,55,54 --rounds 4 --iters 3 || exit 99
for f in zipf full; do grep -h verify_variant "$O/$f.log" | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(sys.argv[1], d["verify_variant"], d["ms_verify_only"])' $f; done | tee "$O/summary.txt"
grep -h GiB_s "$O/c2.log" | tee -a "$O/summary.txt"
