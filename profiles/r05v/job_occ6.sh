#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05w: is r05v's 8-wide loss (+18 % on C, +23 % on E) the occupancy-7 spills?  The 8-wide kernel at occupancy 6
# (32 B/lane of scratch against 56 at 7) against the 4-wide at its default 7.  Prediction: occupancy 6 recovers at most
# 5 points of the 18; the 8-wide tree stays a loss on C.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05w; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u tools/wide8_ab.py --skip-parity --configs C --reps 2 --w8-occupancy 6 > $OUT/ab_occ6.log 2>&1
grep -v '"rep": 0' $OUT/ab_occ6.log | grep speed | cut -c1-200
echo job done
