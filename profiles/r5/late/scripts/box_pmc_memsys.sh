#!/bin/bash
# Memory-pipeline counters of the small-record pipeline (count pass, dense2)
# and of C2's k_full_blocks4 for comparison: L1->L2 request count and latency,
# L1 stalls, TA stalls, L2 hits.  One counter group per rocprofv3 run.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/memsys
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() { "$R/tools/box_step.sh" "$@" || exit 99; }
i=0
for grp in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  step 200 "$O/small_pmc$i.log" rocprofv3 --pmc $grp -d "$O/small/pmc$i" -o pmc -f csv -- python3 $R/tools/c3_legs.py --shapes small --iters 2
  step 200 "$O/c2_pmc$i.log" rocprofv3 --pmc $grp -d "$O/c2/pmc$i" -o pmc -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --e2e-gib 0 --c3-gib 0 --c3-small-gib 0
done
python3 $R/tools/pmc_summary.py $O/small > $O/summary_small.txt
python3 $R/tools/pmc_summary.py $O/c2 > $O/summary_c2.txt
rm -rf $O/small $O/c2
