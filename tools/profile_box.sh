#!/bin/bash
# On-box profiling: kernel-trace stats of bench.py and PMC passes (one
# counter group per rocprofv3 run, never combined with other tracing).
# usage: tools/profile_box.sh <tag> [variant list for PMC]
set -u
tag=$1; variants=${2:-0,100}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
step 120 "$O/counters_list.log" rocprofv3 -L
step 300 "$O/bench_trace.log" rocprofv3 --kernel-trace --stats -d "$O/bench_trace" -o bench -f csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu
W="python3 $R/tools/variants.py --variants $variants --rounds 1 --iters 2"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step 300 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/pmc$i" -o pmc -f csv -- $W
done
echo done > "$O/DONE"
