#!/bin/bash
# r06r: the node rows prefetched inside the first leaf round, after the round's own record loads (so the in-order vmcnt
# lets the round wait for its records only; every lane loads: slots past the end load record 0, lanes without a next
# node load node 0's rows), at 4 waves per SIMD (111 VGPRs, no spills).  Against the same build without the prefetch,
# two alternating runs each on config B, plus frame hashes.  Prediction (r06p's ceiling 12.4 %, minus the iterations
# after a pass): the critical wave's iteration -4 to -8 %; frames identical.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06r; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
for rep in 1 2; do
CRT_HIP_LIB=$LX/occ4/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py --occupancy 4 > $OUT/B_occ4_$rep.json 2> $OUT/B_occ4.err
CRT_HIP_LIB=$LX/occ4pf2/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py --occupancy 4 > $OUT/B_occ4pf2_$rep.json 2> $OUT/B_occ4pf2.err
done
CRT_HIP_LIB=$LX/occ4/libcrt_hip.so timeout -k 10 300 python3 -u tools/frame_hash.py --occupancy 4 > $OUT/hash_occ4.txt 2> $OUT/hash.err
CRT_HIP_LIB=$LX/occ4pf2/libcrt_hip.so timeout -k 10 300 python3 -u tools/frame_hash.py --occupancy 4 > $OUT/hash_occ4pf2.txt 2>> $OUT/hash.err
echo job done
