#!/bin/bash
# Kernel traces of the c3 / c3_small legs with the count pass in 512- or
# 1024-thread workgroups (REVEL_COUNT_WIDE=0/1), alternating processes.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cw2
mkdir -p $O
i=0
for arm in 0 1 0 1; do
  i=$((i+1))
  for shape in zipf small; do
    REVEL_COUNT_WIDE=$arm timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t_${shape}_${arm}_$i -o run -- python3 $R/tools/c3_legs.py --shapes $shape >> $O/legs_${shape}_$arm.log 2>&1
    grep -h 'k_count_hist\|k_scan_order\|k_verify_rows\|dense2\|k_expand_rows' $(find $O/t_${shape}_${arm}_$i -name '*kernel_stats.csv') | cut -d, -f1-4 | sed "s/^/$shape arm$arm run$i /" >> $O/stats.txt
  done
done
