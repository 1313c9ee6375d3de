#!/bin/bash
# Same box: bench.py's c3 leg after its C2 + end-to-end legs (default run), the
# same leg with a short C2 leg and no end-to-end, and tools/bench_c3.py -- is
# bench.py's c3 field slower because of its image or because of the GPU's state
# after the C2 leg?   usage: tools/r3_c3_where.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; mkdir -p "$O"
S=$R/tools/box_step.sh
$S 300 "$O/bench_default.log" python3 "$R/bench.py" --no-cpu || exit 99
$S 300 "$O/bench_short.log" python3 "$R/bench.py" --no-cpu --steps 1 --warmup 1 --e2e-gib 0 || exit 99
$S 300 "$O/bench_c3.log" python3 "$R/tools/bench_c3.py" --variants 0 --rounds 2 --iters 5 --keep-tail || exit 99
$S 300 "$O/bench_default2.log" python3 "$R/bench.py" --no-cpu || exit 99
for f in bench_default bench_short bench_default2; do
  grep -h '^{' "$O/$f.log" | python3 -c '
import json,sys
d=json.loads(sys.stdin.readline()); print(sys.argv[1], "c2", d["value"], "c3_ms", d["c3"]["ms"], "c3_alg_GB_s", d["c3"]["alg_GB_s_rank0"])' $f
done | tee "$O/summary.txt"
grep -h verify_variant "$O/bench_c3.log" | python3 -c '
import json,sys
d=json.loads(sys.stdin.readline()); print("bench_c3 (1 GiB tiled x4 + tail)", d["ms_count_scan_verify"], d["ms_verify_only"])' | tee -a "$O/summary.txt"
