#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06h: the round-6 HEAD (kernel binary byte-identical to round 5's; the source carries two new profiling switches):
# GPU suite, smoke, the default bench line, its rocprofv3 kernel stats, and the headline's PMC passes on the current
# source (so the line's counters_kernel_source_current holds).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06h; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
bash tools/gpu_job.sh check $O
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc
echo job done
