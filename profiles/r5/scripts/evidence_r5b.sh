#!/bin/bash
# Round-5 evidence, part B (part A: evidence_r5a.sh) on one box, every GPU step under its own time limit
# (tools/box_step.sh stops the script on a fault-class exit status):
#   1. the product GPU suite (-m gpu), smoke()
#   2. bench.py (the driver's default command) and a rocprofv3 kernel trace of it
#   3. PMC passes (one counter per rocprofv3 run): C2 (FETCH_SIZE, WRITE_SIZE ->
#      profiles/pmc_c2.json; LDS bank conflicts), the c3 and c3_small pipelines
#      (FETCH_SIZE, WRITE_SIZE -> profiles/pmc_c3.json / pmc_c3_small.json), all
#      for this build's SHA-256; then bench.py again (every roofline.traffic validated)
# usage: profiles/r5/scripts/evidence_r5.sh <tag>
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev5_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  step 120 "$O/c2pmc$i.log" timeout -s KILL 110 rocprofv3 --pmc $grp -d "$O/c2pmc/pmc$i" -o pmc -f csv -- \
      python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 --e2e-gib 0 --c3-gib 0 --c3-small-gib 0
done
step 60 "$O/pmc_c2_summary.log" python3 "$R/tools/pmc_summary.py" "$O/c2pmc" --json "$R/profiles/pmc_c2.json" \
    --blocks 1048576 --kernel "k_full_blocks4<1024, false>"
step 120 "$O/c2lds.log" timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$O/c2lds/pmc1" -o pmc -f csv -- \
    python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 --e2e-gib 0 --c3-gib 0 --c3-small-gib 0
step 60 "$O/pmc_c2lds_summary.log" python3 "$R/tools/pmc_summary.py" "$O/c2lds"
for shp in zipf small; do
  leg=c3; [ $shp = small ] && leg=c3_small
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    step 180 "$O/${leg}pmc$i.log" timeout -s KILL 170 rocprofv3 --pmc $grp -d "$O/${leg}pmc/pmc$i" -o pmc -f csv -- \
        python3 "$R/tools/bench_c3dev.py" --shape $shp --iters 2
  done
  nb=$(grep -o '"image_bytes": [0-9]*' "$O/${leg}pmc1.log" | head -n 1 | grep -o '[0-9]*$')
  step 60 "$O/pmc_${leg}_summary.log" python3 "$R/tools/pmc_summary.py" "$O/${leg}pmc" --pipeline $shp \
      --image-bytes "$nb" --json "$R/profiles/pmc_${leg}.json"
done
cp "$R"/profiles/pmc_c2.json "$R"/profiles/pmc_c3.json "$R"/profiles/pmc_c3_small.json "$O"/ 2>/dev/null
step 420 "$O/bench_validated.log" python3 "$R/bench.py"
echo done > "$O/DONE"
