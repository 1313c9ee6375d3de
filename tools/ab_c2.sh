#!/bin/bash
# A/B of builds of librevel_wal.so on bench.py's C2 leg, alternating processes:
#   tools/ab_c2.sh <tag> <rounds> A.so B.so ...
set -u
tag=$1; n=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag/ab_c2
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for L in "$@"; do
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L").log" python3 "$R/tools/bench_c2dev.py" --lib "$L" || exit 99
  done
done
cat "$O"/run_*.log | grep '^{' | python3 -c '
import json, sys, statistics as st
rows = [json.loads(l) for l in sys.stdin]
for lib in sorted({r["lib"] for r in rows}):
    v = [r["ms"] for r in rows if r["lib"] == lib]
    ok = all(r["all_ok"] and r["stable"] for r in rows if r["lib"] == lib)
    print(lib, "ms", v, "median", round(st.median(v), 4), "frac", round(34364981248 / (st.median(v) / 1e3) / 8e12, 4), "ok", ok)
' | tee "$O/summary.txt"
