#!/bin/bash
# r03aq: config E (1M triangles, 512 spp; variant 8 at occupancy 7) regeneration threshold 44 (default) / 40 / 52.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
E="--scene cornell_1m --spp 512"
bash tools/gpu_job.sh sweep r03aq 2 "T44=$E" "T40=$E --regen-threshold 40" "T52=$E --regen-threshold 52"
