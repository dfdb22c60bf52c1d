#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05aa: the path state only the pass reads (RNG, sum, throughput, counters: 15 words) kept in memory between passes
# (-DCRT_COLD_STATE, lib_exp/cold) so that fewer registers live across the loop: occupancy 8 compiles with 11 VGPR
# spills instead of 19.  Predictions (config C main kernel vs HEAD's occupancy 7): in-tree occ 7 = HEAD (control),
# in-tree occ 8 +15 .. +25 %, cold occ 7 +0 .. +2 %, cold occ 8 -3 .. +5 %.  Frames identical everywhere.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05aa; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/cold/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u tools/cold_ab.py --configs S,C --occupancy 7,8 --reps 2 > $OUT/intree.log 2>&1
grep -v '"rep": 0' $OUT/intree.log | cut -c1-200
CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/cold/libcrt_hip.so CRT_HOST_LIB=raytracer-cuda_amd/lib_exp/cold/libcrt_host.so \
  timeout -k 10 300 python3 -u tools/cold_ab.py --configs S,C --occupancy 7,8 --reps 2 > $OUT/cold.log 2>&1
grep -v '"rep": 0' $OUT/cold.log | cut -c1-200
echo job done
