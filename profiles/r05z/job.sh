#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05z: the GPU suite, smoke, the default bench and a rocprofv3 kernel-stats pass at HEAD (kernel source unchanged since
# r05u; host worker-thread change).  Prediction: 169 passed, bench ~21,2xx Mrays/s.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05z; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_prof.log 2>&1
find $OUT/prof -name "*kernel_stats.csv" | head -2
echo job done
