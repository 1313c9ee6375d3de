#!/bin/bash
# Round-4 evidence on one box, every GPU step under its own time limit
# (tools/box_step.sh stops the script on a fault-class exit status):
#   1. the product GPU suite (-m gpu), smoke(); the experiment arms (-m experiment)
#   2. bench.py (the driver's default command) and a rocprofv3 kernel trace of it
#   3. C2 PMC passes (FETCH_SIZE, WRITE_SIZE) -> profiles/pmc_c2.json for this
#      build's SHA-256, then bench.py again (roofline.traffic validated)
#   4. C3 and c3_small kernel timelines of bench.py's images (tools/bench_c3dev.py)
# usage: tools/evidence_r4.sh <tag>
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 600 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step 120 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step 300 "$O/bench.log" python3 "$R/bench.py"
step 300 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  step 300 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/c2pmc/pmc$i" -o pmc -f csv -- \
      python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 --e2e-gib 0 --c3-gib 0 --c3-small-gib 0
done
step 60 "$O/pmc_summary.log" python3 "$R/tools/pmc_summary.py" "$O/c2pmc" --json "$R/profiles/pmc_c2.json" \
    --blocks 1048576 --kernel "k_full_blocks4<1024, false>"
cp "$R/profiles/pmc_c2.json" "$O/pmc_c2.json"
step 300 "$O/bench_validated.log" python3 "$R/bench.py" --no-cpu
for shp in zipf small; do
  step 300 "$O/tl_$shp.log" rocprofv3 --kernel-trace -d "$O/tl_$shp" -o tl -- python3 "$R/tools/bench_c3dev.py" --shape $shp --iters 5
  python3 "$R/tools/kernel_timeline.py" "$O/tl_$shp" --after k_count_hist > "$O/timeline_$shp.txt" 2>&1
done
step 300 "$O/pytest_experiments.log" python3 -u -m pytest "$R/tests/test_experiments_gpu.py" -m experiment -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider
echo done > "$O/DONE"
