#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06b: PMC passes for the N = 2 / 4 / 8 rank-0 share workloads (1000 / 500 / 250 spp from subsequence 0, one GPU,
# bench.py --share 0 N), so the N > 1 line's roofline has counters of its own workload; then the N = 2 line at full
# size with both ranks on this one GPU (gloo), for its statistical parity field at 2560x1440 x 2000 spp.
# Prediction: per-ray VALU of the shares within 2 % of the 2000-spp frame's 41.2 (the same paths, fewer per pixel);
# the N = 2 parity ratio within 0.95-1.05 on every channel.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06b; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
for n in 2 4 8; do
  bash tools/pmc.sh gpurun_out/$O/pmc_s$n --share 0 $n
done
cd $R
timeout -k 10 600 python3 bench.py --gpus 2 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_n2_gloo.log 2>&1
echo job done
