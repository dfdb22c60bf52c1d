#!/bin/bash
# r06z7: the interactive loop (bin/crt_viewer, 600 frames of 1 spp at 2560x1440, still and orbiting, rebuilt BVH) on the
# final library (variant 7, unchanged kernel; the library gained the occupancy-4 kernel and the probe statistics).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_job.sh viewer r06z7
echo job done
