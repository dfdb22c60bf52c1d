#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05x: the 8-wide tree (profiles/r05v/wide8.patch applied) on config B, the latency-bound frame (one tile's sample chain
# at ~1 us per wave iteration): 45 % fewer node steps per ray shorten the chain's dependent round trips
# even though they cost more issue.  Prediction: B -5 % .. +5 % (8-wide vs 4-wide), occupancy 6 (B's default).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05x; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u tools/wide8_ab.py --skip-parity --configs B --reps 4 > $OUT/ab_B.log 2>&1
grep -v '"rep": 0' $OUT/ab_B.log | grep speed | cut -c1-200
echo job done
