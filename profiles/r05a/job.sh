#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05a: round-5 start: the GPU suite with the new config-E / config-B oracle tests, smoke, the default bench (new
# end-to-end / algorithmic_survey fields) and a one-rank RCCL bench (per-rank render / reduce timings), rocprofv3 stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05a; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --no-cpu-baseline --no-parity > $OUT/bench_rccl1.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity > $OUT/bench_prof.log 2>&1
echo job done
