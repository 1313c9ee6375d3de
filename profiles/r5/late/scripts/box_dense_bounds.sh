#!/bin/bash
# dense2 bound probe: kernel traces of the c3_small leg with the product
# library, a build whose dense2 folds words by XOR instead of the table CRC
# (-DREVEL_DENSE_DIAG=1: the load pipeline alone) and one whose dense2 takes
# register data instead of loads (-DREVEL_DENSE_DIAG=2: the CRC work alone).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dbounds
mkdir -p $O
cp $R/revel_amd/librevel_wal.so $O/product.so
for i in 1 2; do
  for arm in ${ARMS:-product diag1 diag2}; do
    if [ $arm = product ]; then cp $O/product.so $R/revel_amd/librevel_wal.so; else cp $R/build/ab/$arm.so $R/revel_amd/librevel_wal.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t_${arm}_$i -o run -- python3 $R/tools/c3_legs.py --shapes small >> $O/legs_$arm.log 2>&1
  done
done
cp $O/product.so $R/revel_amd/librevel_wal.so
