#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06l: the statistical parity field with the exchangeable control (an independent N-way frame from families
# N..2N-1) for the frame mean: the N = 8 and N = 2 lines over gloo on one GPU, and the bench launch GPU test.
# Prediction: displayed mean z against the other N-way frame below 3 on every channel; RMS ratio unchanged (1.000x).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06l; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dist.py -k "bench_gpus_2 or large_subsequence" -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 900 python3 -u bench.py --gpus 8 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n8_gloo.log 2>&1
timeout -k 10 600 python3 -u bench.py --gpus 2 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n2_gloo.log 2>&1
echo job done
