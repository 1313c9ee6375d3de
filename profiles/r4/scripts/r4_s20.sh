#!/bin/bash
# Round 4, session 20: the product suite on the build whose rows kernel shares
# list positions per workgroup; per-wave end times of the C2 kernel (probe).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s20; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 600 $O/pytest_product.log python3 -u -m pytest $R/tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
ok $O/pytest_product.log || { echo "product tests failed"; tail -40 $O/pytest_product.log; exit 1; }
step 300 $O/c2_wavetime.log python3 $R/tools/c2_wavetime.py --lib $A/c2wt.so
step 300 $O/c2_wavetime2.log python3 $R/tools/c2_wavetime.py --lib $A/c2wt.so
echo done > $O/DONE
