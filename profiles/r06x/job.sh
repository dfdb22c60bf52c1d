#!/bin/bash
# r06x: the occupancy-4 rule on other scenes below the threshold: the 1M-triangle scene at 1280x720 (256 spp) and the
# plain Cornell box at 1280x720 (256 spp), automatic (4) against 6, two rounds (tools/occ_sweep.py).  Prediction: both
# faster at 4, as config B (frames of ~2 tiles per slot end with their sample chains).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06x; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/occ_sweep.py --scene cornell_1m --w 1280 --h 720 --spp 256 --occ 0 6 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
timeout -k 10 300 python3 -u tools/occ_sweep.py --scene cornell --w 1280 --h 720 --spp 256 --occ 0 6 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
echo job done
