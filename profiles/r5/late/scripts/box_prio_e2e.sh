#!/bin/bash
# ADVICE r4 (rotate_prio): C5 replay of a records-layout image with the verify
# kernels' wave-priority rotation on (the product build) and off
# (-DREVEL_DENSE_PRIO=0 -DREVEL_ROWS_PRIO=0, tools/build_variant.sh noprio),
# alternating processes.  The ring loader overlaps window i's verify with
# window i+1's H2D and per-window work on the copy stream.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prio
mkdir -p $O
cp $R/revel_amd/librevel_wal.so $O/prod.so
for i in 1 2 3; do
  for arm in prod noprio; do
    if [ $arm = prod ]; then cp $O/prod.so $R/revel_amd/librevel_wal.so; else cp $R/build/ab/noprio.so $R/revel_amd/librevel_wal.so; fi
    timeout -k 10 200 python3 -u $R/tools/bench_e2e.py --mode records --gib 8 --threads 8 --loader ring,shard --repeat 2 \
        | sed "s/^/$arm run$i /" >> $O/e2e.log
  done
done
cp $O/prod.so $R/revel_amd/librevel_wal.so
