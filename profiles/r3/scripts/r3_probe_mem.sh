#!/bin/bash
# Memory-path probes of k_verify_rows (experiment arms, wrong CRCs for the DIAG
# ones): control 24, no captures 26 / 38 (8- / 16-row ring), loads + XOR only
# 35 / 36 (8- / 16-row ring), no transposes 37; on the Zipf image and on full
# blocks, then C2 on full blocks for reference.   usage: tools/r3_probe_mem.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 300 "$O/zipf.log" python3 "$R/tools/bench_c3.py" --variants 24,35,36,40,41 --rounds 3 --iters 3 || exit 99
$S 300 "$O/full.log" python3 "$R/tools/bench_c3.py" --image full --variants 24,35,36,39,40,41,42 --rounds 3 --iters 3 || exit 99
$S 300 "$O/c2.log" python3 "$R/tools/variants.py" --blocks 131072 --variants 100,0 --rounds 3 --iters 5 || exit 99
for f in zipf full; do grep -h verify_variant "$O/$f.log" | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(sys.argv[1], d["verify_variant"], d["ms_verify_only"], d["physical_records"])' $f; done | tee "$O/summary.txt"
grep -h GiB_s "$O/c2.log" | tee -a "$O/summary.txt"
