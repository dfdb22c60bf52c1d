# r03i: bench.py's own multi-rank path rehearsed on one GPU (gloo; the driver runs nccl = RCCL on an 8-GPU node)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03i; mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 --dist-backend gloo > $OUT/bench_${n}rank_gloo.log 2>&1
  tail -1 $OUT/bench_${n}rank_gloo.log | cut -c1-300
done
