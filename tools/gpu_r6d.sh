#!/bin/bash
# Kernel traces of the Zipf c3 leg: product vs count passes capped at K hops
# (timing probes, wrong counts), to size a capped count pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r6d; mkdir -p $O
cp $R/revel_amd/librevel_wal.so $O/product.so
for arm in prod maxhops16 maxhops24; do
  cp $R/build/ab/lib_$arm.so $R/revel_amd/librevel_wal.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$arm -o trace -- python3 $R/tools/c3_legs.py --shapes zipf --iters 9 > $O/$arm.log 2>&1 || { echo "arm $arm failed"; cp $O/product.so $R/revel_amd/librevel_wal.so; exit 1; }
done
cp $O/product.so $R/revel_amd/librevel_wal.so
echo done
