#!/bin/bash
# r03ae: ablations (timing only, the frames differ): the Lambert/Metal unit-sphere rejection loop and the lens-disk
# rejection loop each cut to one candidate, to bound what a faster rejection sampler could gain.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_job.sh libs r03ae 2 raytracer-cuda_amd/lib_exp/ruv/libcrt_hip.so raytracer-cuda_amd/lib_exp/disk/libcrt_hip.so
