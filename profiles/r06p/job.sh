#!/bin/bash
# r06p: how long the node step waits for its seven rows and the leaf round for its records (-DCRT_PROFILE_ROWS: the
# loads issued, then an explicit vmcnt(0) between two s_memtime), for B's critical wave, B's waves and C at 256 spp.
# Prediction: for the critical wave the row wait is 300-600 of the node step's ~1,800 cycles.  It bounds what any
# node-row prefetch could save on the chain.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06p; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
CRT_HIP_LIB=$LX/passrowscrit/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py --w 1280 --h 720 --spp 256 > $OUT/B_crit.json 2> $OUT/B_crit.err
CRT_HIP_LIB=$LX/passrows/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py --w 1280 --h 720 --spp 256 > $OUT/B_all.json 2> $OUT/B_all.err
CRT_HIP_LIB=$LX/passrows/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py > $OUT/C256_all.json 2> $OUT/C256_all.err
echo job done
