#!/bin/bash
# PMC passes over the C3 verify benchmark (one counter group per rocprofv3 run).
set -u
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c3prof_$tag
mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
W="python3 $R/tools/bench_c3.py --variants ${C3_VARIANT:-0} --iters 2 ${C3_ARGS:-}"
i=0
for grp in "FETCH_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step 300 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/pmc$i" -o pmc -f csv -- $W
done
echo done > "$O/DONE"
