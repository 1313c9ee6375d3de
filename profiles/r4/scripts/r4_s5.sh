#!/bin/bash
# Round 4, session 5: dense2 as the production dense verify kernel (GPU suite
# subset), the count pass with idle-lane prefetch (parity + A/B on bench.py's
# images), the VMM probe's modes in ONE process (the sequence that failed in
# session 3), then the driver's bench command.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s5; mkdir -p $O
export TMPDIR=/tmp
A=$R/build/ab
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
ok() { grep -q " passed" $1 && ! grep -q -E "[0-9]+ failed|[0-9]+ error" $1; }
step 400 $O/pytest_verify.log python3 -u -m pytest $R/tests/test_gpu.py $R/tests/test_gpu_guard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or expander or dense or count or guard or unmapped or append"
ok $O/pytest_verify.log || { echo "tests failed"; tail -40 $O/pytest_verify.log; exit 1; }
REVEL_LIB=$A/countpf.so step 400 $O/pytest_countpf.log python3 -u -m pytest $R/tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "verify or count or expander"
ok $O/pytest_countpf.log || { echo "countpf tests failed"; tail -40 $O/pytest_countpf.log; exit 1; }
$R/tools/ab_dev.sh r4s5 3 zipf $A/base.so:0 $A/countpf.so:0 || exit 99
$R/tools/ab_dev.sh r4s5 2 small $A/base.so:0 $A/countpf.so:0 || exit 99
for L in base countpf; do
  step 300 $O/tl_$L.log rocprofv3 --kernel-trace -d $O/tl_$L -o tl -- python3 $R/tools/bench_c3dev.py --lib $A/$L.so --walk 0 --iters 3
  python3 $R/tools/kernel_timeline.py $O/tl_$L --after k_count_hist | tail -6 > $O/timeline_$L.txt 2>&1
done
step 300 $O/vmm_all.log python3 -u $R/tools/vmm_probe.py --iters 20 --modes nosync,sync,keepva,keepphys,plain
step 400 $O/bench.log python3 $R/bench.py
echo done > $O/DONE
