#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04w: verification at the round-4 HEAD as the driver runs it: the GPU suite, smoke, the default bench, and the RCCL
# one-rank bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04w; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -2 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29516 bench.py --gpus 1 --steps 3 --warmup 1 > $OUT/bench_rccl1.log 2>&1
tail -1 $OUT/bench_rccl1.log | cut -c1-200
echo job done
