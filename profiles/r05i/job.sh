#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05i: the benches of the r05h final set again, with profiles/roofline_counters.json summarised from the timed
# dispatch only (r05h's on-box summary had added the end-to-end leg's frame in).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05i; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py profiles/roofline_counters.json > $OUT/sha.txt
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python3 bench.py --width 1280 --height 720 --spp 256 --steps 5 --no-cpu-baseline > $OUT/B.log 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline > $OUT/E.log 2>&1
timeout -k 10 300 python3 bench.py --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --cpu-threads 1 > $OUT/A.log 2>&1
for f in B E A; do echo "$f: $(tail -1 $OUT/$f.log | cut -c1-160)"; done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29514 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/bench_rccl1.log 2>&1
tail -1 $OUT/bench_rccl1.log | cut -c1-200
echo job done
