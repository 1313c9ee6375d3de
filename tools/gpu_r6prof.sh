#!/bin/bash
# Kernel trace + memory-system PMC passes of the c3_small leg for two
# libraries (product tree lib = arm "a", arg = arm "b"):  tools/gpu_r6prof.sh <tag> <b.so>
set -u
tag=$1; blib=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag; mkdir -p "$O"
export TMPDIR=/tmp
cp "$R/revel_amd/librevel_wal.so" "$O/a.so"
step() { "$R/tools/box_step.sh" "$@" || { cp "$O/a.so" "$R/revel_amd/librevel_wal.so"; exit 99; }; }
W="python3 $R/tools/c3_legs.py --shapes small --iters 3 --warmup-calls 3"
for arm in a b; do
  [ $arm = b ] && cp "$blib" "$R/revel_amd/librevel_wal.so"
  step 240 "$O/${arm}_trace.log" rocprofv3 --kernel-trace --stats -d "$O/${arm}_trace" -o tr -- $W
  i=0
  for grp in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" \
             "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUFFER_READ_WAVEFRONTS_sum" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
    i=$((i+1))
    step 120 "$O/${arm}_pmc$i.log" rocprofv3 --pmc $grp -d "$O/${arm}_pmc/pmc$i" -o pmc -f csv -- $W
  done
  python3 "$R/tools/pmc_summary.py" "$O/${arm}_pmc" > "$O/${arm}_summary.txt" 2>&1
  python3 "$R/tools/kernel_durations.py" "$O/${arm}_trace" verify_records_dense > "$O/${arm}_dense_durs.txt" 2>&1
done
cp "$O/a.so" "$R/revel_amd/librevel_wal.so"
rm -f "$O/a.so"
echo done
