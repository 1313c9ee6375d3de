#!/bin/bash
# Round evidence on the box: bench line, rocprofv3 kernel-trace stats of the
# SAME bench command, PMC passes (one counter group per run) over the C2
# launches alone and over the C3 verify, C3 throughput + its kernel trace.
# usage: tools/evidence_box.sh <tag>
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 300 "$O/bench.log" python3 "$R/bench.py"
step 300 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py"
CGROUPS=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
        "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum")
i=0
for grp in "${CGROUPS[@]}"; do
  i=$((i+1))
  # C2 launches only (no end-to-end / C3 legs mixed into the per-kernel means)
  step 300 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/pmc$i" -o pmc -f csv -- \
      python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 --e2e-gib 0 --c3-gib 0
  step 300 "$O/c3pmc$i.log" rocprofv3 --pmc $grp -d "$O/c3pmc/pmc$i" -o pmc -f csv -- \
      python3 "$R/tools/bench_c3.py" --variants 0 --iters 2
done
step 300 "$O/c3.log" python3 "$R/tools/bench_c3.py"
step 300 "$O/c3_trace.log" rocprofv3 --kernel-trace --stats -d "$O/c3_trace" -o c3 -f csv -- python3 "$R/tools/bench_c3.py" --iters 3
echo done > "$O/DONE"
