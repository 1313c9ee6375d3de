#!/bin/bash
# Kernel trace (per-kernel stats) and two SQ PMC passes of tools/bench_c3.py
# for each given build: tools/r3_trace_ab.sh <tag> A.so [B.so ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$R/gpurun_out/$tag; mkdir -p "$O"
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
for L in "$@"; do
  b=$(basename "$L" .so)
  W="python3 $R/tools/bench_c3.py --lib $L --variants 0 --rounds 1 --iters 3"
  mkdir -p "$O/$b"
  step 300 "$O/$b/trace.log" rocprofv3 --kernel-trace --stats -d "$O/$b/trace" -o trace -f csv -- $W
  step 300 "$O/$b/pmcA.log" rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$O/$b/pmcA" -o pmc -f csv -- $W
  step 300 "$O/$b/pmcB.log" rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
      SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d "$O/$b/pmcB" -o pmc -f csv -- $W
done
echo done > "$O/DONE"
