#!/bin/bash
# dense2 load-pattern probes (loads + XOR fold, wrong CRCs): DIAG 1 = the
# product's lane-owned loads, 4 = lane pairs each loading one 64-B sector of
# the same 128-B lines, 5 = each lane its own 128-B aligned line.  Kernel time
# and L1->L2 request count per build.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sector
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
cp $R/revel_amd/librevel_wal.so $O/product.so
for arm in diag1 diag4 diag5; do
  cp $R/build/ab/$arm.so $R/revel_amd/librevel_wal.so
  step 200 "$O/${arm}_trace.log" rocprofv3 --kernel-trace -d "$O/t_$arm" -o run -- python3 $R/tools/c3_legs.py --shapes small
  step 200 "$O/${arm}_pmc.log" rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum -d "$O/p_$arm/pmc1" -o pmc -f csv -- python3 $R/tools/c3_legs.py --shapes small --iters 2
  python3 $R/tools/pmc_summary.py "$O/p_$arm" > "$O/${arm}_pmc_summary.txt"
  rm -rf "$O/p_$arm"
done
cp $O/product.so $R/revel_amd/librevel_wal.so
