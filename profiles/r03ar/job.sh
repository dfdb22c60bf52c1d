#!/bin/bash
# r03ar: config B (1280x720, 256 spp; 2 tiles per wave slot) at occupancy 6 (default) against 5.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
B="--width 1280 --height 720 --spp 256 --steps 5"
bash tools/gpu_job.sh sweep r03ar 3 "occ6=$B" "occ5=$B --occupancy 5"
