#!/bin/bash
# Kernel trace (per-kernel stats) of tools/bench_c3.py for each given build:
#   tools/r3_trace_only.sh <tag> A.so [B.so ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/$tag; mkdir -p "$O"
export TMPDIR=/tmp
for L in "$@"; do
  b=$(basename "$L" .so)
  mkdir -p "$O/$b"
  "$R/tools/box_step.sh" 300 "$O/$b/trace.log" rocprofv3 --kernel-trace --stats -d "$O/$b/trace" -o trace -f csv -- \
      python3 "$R/tools/bench_c3.py" --lib "$L" --variants 0 --rounds 1 --iters 5 || exit 99
  f=$(find "$O/$b/trace" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$b" <<'PY' | tee -a "$O/summary.txt"
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print(sys.argv[2], n[:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
done
