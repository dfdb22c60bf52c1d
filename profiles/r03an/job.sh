#!/bin/bash
# r03an: at the occupancy-7 HEAD: variant 8's critical tiles (count) re-swept on config C, and variant 10's regeneration
# threshold at its new occupancy 6 (reference-BVH config C).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_job.sh sweep r03an 2 "crit_auto=" "crit512=--critical-tiles 512" "crit2048=--critical-tiles 2048" "crit0=--critical-tiles 0"
bash tools/gpu_job.sh sweep r03an_v10 2 "T24=--bvh reference --steps 2" "T20=--bvh reference --steps 2 --regen-threshold 20" "T32=--bvh reference --steps 2 --regen-threshold 32"
