#!/bin/bash
# r03y: regeneration threshold and config B's critical lanes re-swept with the root step in the pass (top levels 1).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/gpu_job.sh sweep r03y 2 "T44=--regen-threshold 44" "T40=--regen-threshold 40" "T48=--regen-threshold 48" \
  "T52=--regen-threshold 52"
B="--width 1280 --height 720 --spp 256"
bash tools/gpu_job.sh sweep r03y_B 2 "c16=$B --critical-lanes 16" "c8=$B --critical-lanes 8" "c24=$B --critical-lanes 24"
