#!/bin/bash
# Kernel trace + PMC passes of the staged dense kernel (arm $2, default 6) beside dense2 on
# the c3_small image (tools/dense_staged_ab.py, one round):  tools/gpu_r6stprof.sh <tag> [arm]
set -u
tag=$1; arm=${2:-6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag; mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
W="python3 $R/tools/dense_staged_ab.py --shapes small --arms $arm --rounds 1 --iters 2 --warmup 1"
step 240 "$O/trace.log" rocprofv3 --kernel-trace --stats -d "$O/trace" -o tr -- $W
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step 120 "$O/pmc$i.log" rocprofv3 --pmc $grp -d "$O/pmc/pmc$i" -o pmc -f csv -- $W
done
python3 "$R/tools/pmc_summary.py" "$O/pmc" > "$O/summary.txt" 2>&1
python3 "$R/tools/kernel_durations.py" "$O/trace" verify_records_dense > "$O/dense_durs.txt" 2>&1
cat "$O/summary.txt" "$O/dense_durs.txt"
