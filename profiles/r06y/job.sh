#!/bin/bash
# r06y: calibration of the probe-based occupancy choice (rho = largest tile work / mean work per occupancy-6 wave slot):
# rho and the main kernel at the automatic choice, at 4 and at 6, for frames on both sides of the chain-bound line.
# Prediction: the frames where 4 won in r06t-r06x have rho above the ones where 6 won, with a gap to put CRT_CHAIN_RHO in.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06y; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
S="timeout -k 10 300 python3 -u tools/occ_sweep.py --occ 0 4 6"
for spec in "cornell_bunny 1280 720 256" "cornell 1280 720 256" "cornell_1m 1280 720 256" "cornell_bunny 1280 800 256" \
            "cornell_bunny 1366 768 256" "cornell_bunny 1440 810 256" "cornell_bunny 1600 900 256" \
            "cornell_bunny 640 360 256" "cornell 640 360 256" "cornell_1m 640 360 256"; do
  set -- $spec
  $S --scene $1 --w $2 --h $3 --spp $4 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
done
$S --w 2560 --h 1440 --spp 2000 --pixel-shard 0 8 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
echo job done
