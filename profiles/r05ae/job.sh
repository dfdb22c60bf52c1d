#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05ae: the root's internal children in LDS too (-DCRT_TOP_LEVELS=2, lib_exp/top2; crt_renderer_set_top_levels 1 vs 2
# in the same binary) on config B, whose frame is one tile's chain of dependent round trips (one fewer per ray at
# level 2), and C (measured in round 3 at +4.9 %).  Predictions: B -2 .. -6 % at level 2; C +2 .. +5 %; frames identical.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05ae; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
T="CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/top2/libcrt_hip.so CRT_HOST_LIB=raytracer-cuda_amd/lib_exp/top2/libcrt_host.so"
env $T timeout -k 10 400 python3 -u tools/cold_ab.py --configs B,C --occupancy 0 --top-levels 1,2 --reps 3 > $OUT/top2.log 2>&1
grep -v '"rep": 0' $OUT/top2.log | cut -c1-200
echo job done
