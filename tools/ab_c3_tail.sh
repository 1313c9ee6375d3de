#!/bin/bash
# A/B of two builds of librevel_wal.so on the C3 image with and without the
# writer's partial tail block, alternating processes:
#   tools/ab_c3_tail.sh <tag> A.so B.so [rounds]
set -u
tag=$1; A=$2; B=$3; n=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab_$tag
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for L in "$A" "$B"; do
    for T in "" "--keep-tail"; do
      "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L")${T}.log" \
          python3 "$R/tools/bench_c3.py" --lib "$L" --variants 0 --rounds 2 --iters 5 $T || exit 99
    done
  done
done
grep -h '"verify_variant"' "$O"/run_*.log | python3 -c '
import json, sys, statistics as st
rows = [json.loads(l) for l in sys.stdin]
for lib in sorted({r["lib"] for r in rows}):
  for tail in (False, True):
    rr = [r for r in rows if r["lib"] == lib and ("partial tail" in r["workload"]) == tail]
    v = [r["ms_verify_only"] for r in rr]
    t = [r["ms_count_scan_verify"] for r in rr]
    ok = all(r["matches_production"] and r["bad_records"] == 0 for r in rr)
    print(lib, "tail" if tail else "whole", "verify_ms", [round(x, 4) for x in v], "median", round(st.median(v), 4),
          "total_median", round(st.median(t), 4), "ok", ok)
' | tee "$O/summary.txt"
