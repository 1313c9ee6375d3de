cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5b
timeout -k 10 200 python -u tools/fused_phases.py --lib build/ab/phases.so --shape small > gpurun_out/r5b/phases_small.log 2>&1 && \
timeout -k 10 200 python -u tools/fused_phases.py --lib build/ab/phases.so --shape zipf > gpurun_out/r5b/phases_zipf.log 2>&1
rc=$?; echo rc=$rc; cat gpurun_out/r5b/*.log | tail -6
