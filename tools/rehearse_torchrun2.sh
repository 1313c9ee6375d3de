set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4tr; mkdir -p $O
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  "$R/bench.py" --gpus 2 --steps 10 --warmup 2 > "$O/torchrun2.log" 2>&1
echo "rc=$?" >> "$O/torchrun2.log"
