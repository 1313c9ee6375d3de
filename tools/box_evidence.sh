#!/bin/bash
# Evidence for the build in this tree, on one MI355X box (run through gpurun):
#   smoke, the product GPU suite, PMC FETCH_SIZE / WRITE_SIZE passes of the C2
#   kernel and of the c3 / c3_small pipelines (-> profiles/pmc_*.json in the
#   box's tree, so the bench below prints validated `traffic`; copies under
#   gpurun_out/<tag>/ to commit), bench.py's default line, and a kernel trace
#   of the c3 legs.  Every GPU step runs under its own time limit; a fault-class
#   exit stops the script (tools/box_step.sh).
# usage: tools/box_evidence.sh <tag>
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 120 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step 600 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider
# PMC: one counter per rocprofv3 run, kernel trace off (gpurun rules)
C2="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --e2e-gib 0 --c3-gib 0 --c3-small-gib 0"
step 300 "$O/pmc_c2_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$O/c2pmc/pmc1" -o pmc -f csv -- $C2
step 300 "$O/pmc_c2_write.log" rocprofv3 --pmc WRITE_SIZE -d "$O/c2pmc/pmc2" -o pmc -f csv -- $C2
step 60 "$O/pmc_c2_summary.log" python3 "$R/tools/pmc_summary.py" "$O/c2pmc" --json "$R/profiles/pmc_c2.json"
for shape in zipf small; do
  L="python3 $R/tools/c3_legs.py --shapes $shape --iters 2 --warmup-calls 0"
  step 300 "$O/pmc_${shape}_fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$O/${shape}pmc/pmc1" -o pmc -f csv -- $L
  step 300 "$O/pmc_${shape}_write.log" rocprofv3 --pmc WRITE_SIZE -d "$O/${shape}pmc/pmc2" -o pmc -f csv -- $L
done
ZB=$(grep -h -o '"image_bytes": [0-9]*' "$O"/pmc_zipf_fetch.log | head -1 | grep -o '[0-9]*$')
SB=$(grep -h -o '"image_bytes": [0-9]*' "$O"/pmc_small_fetch.log | head -1 | grep -o '[0-9]*$')
step 60 "$O/pmc_c3_summary.log" python3 "$R/tools/pmc_summary.py" "$O/zipfpmc" --pipeline zipf --image-bytes "$ZB" \
    --json "$R/profiles/pmc_c3.json"
step 60 "$O/pmc_c3_small_summary.log" python3 "$R/tools/pmc_summary.py" "$O/smallpmc" --pipeline small \
    --image-bytes "$SB" --json "$R/profiles/pmc_c3_small.json"
cp "$R"/profiles/pmc_c2.json "$R"/profiles/pmc_c3.json "$R"/profiles/pmc_c3_small.json "$O/"
step 900 "$O/bench.log" python3 "$R/bench.py"
step 300 "$O/c3_trace.log" rocprofv3 --kernel-trace --stats -d "$O/c3_trace" -o c3 -f csv -- \
    python3 "$R/tools/c3_legs.py"
rm -rf "$O/c2pmc" "$O/zipfpmc" "$O/smallpmc"
echo done > "$O/DONE"
