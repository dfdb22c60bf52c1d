#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05af: config B at occupancy 5 against its automatic 6 (HEAD): B's frame is its slowest tile's sample chain, which
# shares its SIMD with the other waves for most of the frame; fewer waves per SIMD give it a larger issue share while
# the rest of the frame has slack.  Prediction: -3 .. +5 %; frames identical.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05af; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u tools/cold_ab.py --configs B --occupancy 6,5 --reps 4 > $OUT/B_occ.log 2>&1
grep -v '"rep": 0' $OUT/B_occ.log | cut -c1-200
echo job done
