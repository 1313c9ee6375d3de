#!/bin/bash
# A/B of builds of librevel_wal.so on bench.py's device-framed c3 image,
# alternating processes so that clock drift spreads over all builds:
#   tools/ab_dev.sh <tag> <rounds> <shape> A.so[:walk] B.so[:walk] ...
# (":1" / ":0" after a library: the fused pipeline on / off in that run)
set -u
tag=$1; n=$2; shape=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag/ab_$shape
mkdir -p "$O"
for i in $(seq 1 "$n"); do
  for spec in "$@"; do
    L=${spec%%:*}; W=""; [ "$spec" != "$L" ] && W="--walk ${spec##*:}"
    "$R/tools/box_step.sh" 300 "$O/run_${i}_$(basename "$L")${W// /}.log" \
        python3 "$R/tools/bench_c3dev.py" --lib "$L" --shape "$shape" --iters 7 $W || exit 99
  done
done
cat "$O"/run_*.log | grep '^{' | python3 -c '
import json, sys, statistics as st
rows = [json.loads(l) for l in sys.stdin]
for lib in sorted({r["lib"] for r in rows}):
    v = [r["ms_median"] for r in rows if r["lib"] == lib]
    w = [r["ms_stream"] for r in rows if r["lib"] == lib and r.get("ms_stream")]
    ok = all(r["bad_records"] == 0 for r in rows if r["lib"] == lib)
    print(lib, "ms", [round(x, 4) for x in v], "median", round(st.median(v), 4),
          "stream", [round(x, 4) for x in w], "median", round(st.median(w), 4) if w else None, "ok", ok)
' | tee "$O/summary.txt"
