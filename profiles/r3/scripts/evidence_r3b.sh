#!/bin/bash
# Round-3 evidence on one box, in two parts (each under gpurun's 20-minute
# limit); every GPU step under its own time limit (tools/box_step.sh stops the
# script on a fault-class exit status).
#   part 1: the product GPU suite, the experiment arms, smoke(), bench.py and a
#           rocprofv3 kernel trace of it, the C2 PMC passes (FETCH_SIZE,
#           WRITE_SIZE) -> profiles/pmc_c2.json (kernel symbol + this build's
#           SHA-256), then bench.py again (roofline.traffic validated, printed)
#   part 2: C3 PMC passes + kernel trace of tools/bench_c3.py, the C3 A/B line,
#           C1 through the native C-ABI driver, C2 vs the streaming-read ceiling
# usage: tools/evidence_r3b.sh <tag> <1|2>
set -u
tag=$1; part=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
if [ "$part" = 1 ]; then
step 900 "$O/pytest_product.log" python3 -u -m pytest "$R/tests" -m gpu -v --timeout 300 --timeout-method thread \
    --ignore="$R/tests/test_experiments_gpu.py"
step 300 "$O/pytest_experiments.log" python3 -u -m pytest "$R/tests/test_experiments_gpu.py" -m gpu -q --timeout 120 \
    --timeout-method thread
step 120 "$O/smoke.log" python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()"
step 300 "$O/bench.log" python3 "$R/bench.py"
step 300 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  step 300 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/c2pmc/pmc$i" -o pmc -f csv -- \
      python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 --e2e-gib 0 --c3-gib 0
done
step 60 "$O/pmc_summary.log" python3 "$R/tools/pmc_summary.py" "$O/c2pmc" --json "$R/profiles/pmc_c2.json" \
    --blocks 1048576 --kernel "k_full_blocks4<1024, false>"
cp "$R/profiles/pmc_c2.json" "$O/pmc_c2.json"
step 300 "$O/bench_validated.log" python3 "$R/bench.py" --no-cpu
echo done > "$O/DONE1"
else
i=0
for grp in "FETCH_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step 300 "$O/c3pmc$i.log" rocprofv3 --pmc $grp -d "$O/c3pmc/pmc$i" -o pmc -f csv -- \
      python3 "$R/tools/bench_c3.py" --variants 0 --iters 2
done
step 300 "$O/c3_trace.log" rocprofv3 --kernel-trace --stats -d "$O/c3_trace" -o c3 -f csv -- \
    python3 "$R/tools/bench_c3.py" --variants 0 --iters 3
step 300 "$O/c3.log" python3 "$R/tools/bench_c3.py" --variants 0,15 --rounds 3 --iters 3
step 120 "$O/c1_native.log" "$R/tools/c1_native" 5
step 300 "$O/c2_vs_ceiling.log" python3 "$R/tools/variants.py" --variants 100,0 --rounds 3 --iters 3
echo done > "$O/DONE2"
fi
