#!/bin/bash
# A/B of librevel_wal.so builds (and REVEL_* switches) on bench.py's c3 / c3_small
# legs, alternating processes: each arm is "<name>=<path to .so>[:ENV=VAL]"; the
# arm's library is copied over revel_amd/librevel_wal.so in the box's tree for its
# run (the product library is restored at the end).
#   tools/ab_libs_c3.sh <tag> <rounds> arm...
set -u
tag=$1; n=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cp "$R/revel_amd/librevel_wal.so" "$O/product.so"
for i in $(seq 1 "$n"); do
  for arm in "$@"; do
    name=${arm%%=*}; rest=${arm#*=}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    [ "$lib" = product ] && lib=$O/product.so
    cp "$lib" "$R/revel_amd/librevel_wal.so"
    env $envs timeout -k 10 200 python3 -u "$R/tools/c3_legs.py" > "$O/run_${i}_$name.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "arm $name rc=$rc"; cp "$O/product.so" "$R/revel_amd/librevel_wal.so"; exit 99; }
    sed "s/^/$name /" "$O/run_${i}_$name.log" | grep shape >> "$O/all.log"
  done
done
cp "$O/product.so" "$R/revel_amd/librevel_wal.so"
python3 - "$O/all.log" <<'PY'
import json, sys, collections, statistics as st
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    name, js = line.split(" ", 1)
    r = json.loads(js)
    d[(r["shape"], name)].append((r["ms_steady_median"], r["ms_isolated_median"], r["bad"], r["nphys"]))
for (shape, name), v in sorted(d.items()):
    print(shape, name, "steady", [x[0] for x in v], "median %.4f" % st.median(x[0] for x in v),
          "isolated median %.4f" % st.median(x[1] for x in v), "bad", sum(x[2] for x in v), "nphys", v[0][3])
PY
