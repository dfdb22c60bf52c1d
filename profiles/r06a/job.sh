#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06a: the GPU suite (with the new bench --gpus 2 launch test), smoke, the default bench line and its rocprofv3
# kernel stats, after the round-5 tree cleanup (stray code objects removed).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06a; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
bash tools/gpu_job.sh check $O
echo job done
