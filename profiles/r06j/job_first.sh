#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06j: the N = 8 path end to end on the one GPU this pool gives: `python bench.py --gpus 8 --dist-backend gloo`
# (no launcher environment: bench.py starts torch.distributed.run with 8 ranks itself; the 8 ranks time-share cuda:0,
# so the timings are not a scaling figure).  Checks: n_gpus 8, eight per-rank render / reduce times, the 250-spp share
# roofline from its own counters, and the statistical parity field, whose expected RMS is sqrt(2) x noise x
# sqrt(1 - 1/8).  Prediction: rms_over_expected within 0.97-1.03 on every channel.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06j; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u bench.py --gpus 8 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n8_gloo.log 2>&1
echo job done
