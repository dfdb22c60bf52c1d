#!/bin/bash
# r06w: config B's schedule knobs re-swept for the occupancy-4 prefetch kernel (they were tuned at occupancy 6): the
# critical tiles' threshold (16 default: 8, 12, 24), their count (1,024 default: 512, 2,048) and the regeneration
# threshold (44: 40, 48), two rounds.  Prediction: within +-1 % of the default except threshold 8 (slower).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BA="--width 1280 --height 720 --spp 256 --steps 3 --warmup 1"
bash tools/gpu_job.sh sweep r06w 2 "def=$BA" "cl8=$BA --critical-lanes 8" "cl12=$BA --critical-lanes 12" \
  "cl24=$BA --critical-lanes 24" "ct512=$BA --critical-tiles 512" "ct2048=$BA --critical-tiles 2048" \
  "rt40=$BA --regen-threshold 40" "rt48=$BA --regen-threshold 48" > gpurun_out/r06w_summary.txt 2>&1
mv gpurun_out/r06w_summary.txt gpurun_out/r06w/summary.txt
echo job done
