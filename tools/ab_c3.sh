#!/bin/bash
# A/B of builds of librevel_wal.so on the C3 image, alternating processes so
# that clock drift spreads over all of them:
#   tools/ab_c3.sh <tag> <rounds> A.so B.so [C.so ...]
set -u
tag=$1; n=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag/ab
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for L in "$@"; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L").log" \
        python3 "$R/tools/bench_c3.py" --lib "$L" --variants 0 --rounds 2 --iters 5 || exit 99
  done
done
grep -h '"verify_variant"' "$O"/run_*.log | python3 -c '
import json, sys, statistics as st
rows = [json.loads(l) for l in sys.stdin]
for lib in sorted({r["lib"] for r in rows}):
    v = [r["ms_verify_only"] for r in rows if r["lib"] == lib]
    t = [r["ms_count_scan_verify"] for r in rows if r["lib"] == lib]
    ok = all(r["matches_production"] and r["bad_records"] == 0 for r in rows if r["lib"] == lib)
    print(lib, "verify_ms", [round(x, 4) for x in v], "median", round(st.median(v), 4),
          "total", [round(x, 4) for x in t], "total_median", round(st.median(t), 4), "ok", ok)
' | tee "$O/summary.txt"
