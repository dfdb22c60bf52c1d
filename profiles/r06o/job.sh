#!/bin/bash
# r06o: config B's critical chain with the next node's rows loaded one leaf round ahead (-DCRT_PREFETCH_EXP), at 4
# waves per SIMD (-DCRT_OCC4_EXP: 109 VGPRs, no spills; the same build without the prefetch: 85 at occupancy 4's
# budget).  Per-iteration time of the critical wave and the frame, both libraries at occupancy 4, plus the default
# library's rule (occupancy 6) for the longest-wave list.  Prediction: the critical wave's iteration -8 to -15 % with
# the prefetch (r06n: the node step is 1,795 of 5,306 cycles, roughly half of it waiting on the rows); frames identical.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06o; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
CRT_HIP_LIB=$LX/crit/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py > $OUT/B_occ6.json 2> $OUT/B_occ6.err
for rep in 1 2; do
CRT_HIP_LIB=$LX/occ4/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py --occupancy 4 > $OUT/B_occ4_$rep.json 2> $OUT/B_occ4.err
CRT_HIP_LIB=$LX/occ4pf/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py --occupancy 4 > $OUT/B_occ4pf_$rep.json 2> $OUT/B_occ4pf.err
done
CRT_HIP_LIB=$LX/occ4/libcrt_hip.so timeout -k 10 300 python3 -u tools/frame_hash.py --occupancy 4 > $OUT/hash_occ4.txt 2> $OUT/hash.err
CRT_HIP_LIB=$LX/occ4pf/libcrt_hip.so timeout -k 10 300 python3 -u tools/frame_hash.py --occupancy 4 > $OUT/hash_occ4pf.txt 2>> $OUT/hash.err
echo job done
