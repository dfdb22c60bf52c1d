#!/bin/bash
# r06u: the occupancy rule's crossover near 4 tiles per occupancy-4 slot (16,384 tiles on 256 CUs): 1280x800 (16,000
# tiles, automatic 4), 1366x768 (16,416, automatic 6), 1440x810 (18,360, automatic 6), each at 4 and 6; and a pixel-shard
# frame (config C, shard 0 of 8: 7,200 tiles at 2000 spp, automatic 4) at 4, 6 and 7.  tools/occ_sweep.py, two rounds.
# Prediction: 1280x800 about even; 1366x768 and 1440x810 faster at 6; the pixel shard (chain-bound) faster at 4.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06u; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
for wh in "1280 800" "1366 768" "1440 810"; do
  set -- $wh
  timeout -k 10 300 python3 -u tools/occ_sweep.py --w $1 --h $2 --spp 256 --occ 4 6 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
done
timeout -k 10 300 python3 -u tools/occ_sweep.py --w 2560 --h 1440 --spp 2000 --occ 0 6 7 --pixel-shard 0 8 >> $OUT/sweep.jsonl 2>> $OUT/sweep.err
echo job done
