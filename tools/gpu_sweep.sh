#!/bin/bash
# Environment sweep of bench.py (GPU box, repo root): one bench run per value of an environment variable, in rounds.
#   tools/gpu_sweep.sh OUT VAR "v1 v2 ..." ROUNDS [bench args]
# Every run has its own time limit; set -e ends the sweep at the first failure.
set -e
OUT=gpurun_out/$1; VAR=$2; VALS=$3; N=$4; shift 4
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity "$@" > $OUT/${VAR}_${v}_$i.log 2>&1
    echo "$VAR=$v round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/${VAR}_${v}_$i.log)"
  done
done
