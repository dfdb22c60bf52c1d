#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05z (second call): the rocprofv3 kernel-stats pass in CSV (the first call wrote the rocpd database only).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05z; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_csv -o bench -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_prof_csv.log 2>&1
find $OUT/prof_csv -name "*kernel_stats.csv"
echo job done
