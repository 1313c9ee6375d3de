#!/bin/bash
# Round 4, session 10: production = captures carried across blocks + the
# expander's three loads in one round trip.  The whole product GPU suite on
# it, the verify tests on the no-carry build (REVEL_CAP_CARRY=0, its batch
# packing fixed), A/B of prev / nocarry / in-tree on both bench images; the
# dense kernel with the 16 B a lane's stream does not reach addressed out of
# range (oob: no fetch) on the small-record image.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s10; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 600 $O/pytest_product.log python3 -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
ok $O/pytest_product.log || { echo "product tests failed"; tail -40 $O/pytest_product.log; exit 1; }
REVEL_LIB=$A/nocarry.so step 400 $O/pytest_nocarry.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander or append"
ok $O/pytest_nocarry.log || { echo "nocarry tests failed"; tail -40 $O/pytest_nocarry.log; exit 1; }
$R/tools/ab_dev.sh r4s10 4 zipf $A/prev.so $A/nocarry.so $R/revel_amd/librevel_wal.so || exit 99
REVEL_LIB=$A/oob.so step 400 $O/pytest_oob.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or dense or guard or unmapped"
ok $O/pytest_oob.log || { echo "oob tests failed"; tail -40 $O/pytest_oob.log; exit 1; }
$R/tools/ab_dev.sh r4s10 3 small $A/prev.so $R/revel_amd/librevel_wal.so $A/oob.so || exit 99
step 300 $O/tl.log rocprofv3 --kernel-trace -d $O/tl -o tl -- python3 $R/tools/bench_c3dev.py --iters 5
python3 $R/tools/kernel_timeline.py $O/tl --after k_count_hist | tail -6 > $O/timeline.txt 2>&1
echo done > $O/DONE
