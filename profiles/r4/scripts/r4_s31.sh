#!/bin/bash
# Round 4, session 31: PMC passes (final build) (one counter group per rocprofv3 run) of the
# current build's C3 kernels on bench.py's Zipf and small-record images.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s31; mkdir -p $O
export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
for shp in small zipf; do
  i=0
  for grp in "FETCH_SIZE" \
             "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_INSTS_SALU" \
             "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    step 300 "$O/${shp}_pmc$i.log" timeout -s KILL 200 rocprofv3 --pmc $grp -d "$O/$shp/pmc$i" -o pmc -f csv -- python3 $R/tools/bench_c3dev.py --shape $shp --iters 2
  done
  python3 $R/tools/pmc_summary.py $O/$shp > $O/summary_$shp.txt 2>&1
done
echo done > $O/DONE
