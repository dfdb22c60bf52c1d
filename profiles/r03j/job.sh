# r03j: pixel sharding (bit-exact multi-GPU mode): GPU suite, default bench, bench.py --shard pixels on 2 gloo ranks
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03j; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29602 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --shard pixels > $OUT/bench_2rank_pixels.log 2>&1
tail -1 $OUT/bench_2rank_pixels.log | cut -c1-300
