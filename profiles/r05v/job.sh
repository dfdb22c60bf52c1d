#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05v: the 8-wide node A/B (round-4 verdict item 4).  Prediction (census x measured visits): main kernel
# on C within -3 % .. +3 % of the 4-wide tree, E +0 .. +6 % (slower: +13 % triangle tests, 56 B/lane of spills at
# occupancy 7 against 16).  Frames bit-identical between the trees.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05v; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u tools/wide8_ab.py --parity-only > $OUT/parity.log 2>&1
tail -2 $OUT/parity.log | cut -c1-300
timeout -k 10 600 python3 -u tools/wide8_ab.py --configs C,E --reps 3 > $OUT/ab.log 2>&1
grep -v '"rep": 0' $OUT/ab.log | grep speed | cut -c1-220
echo job done
