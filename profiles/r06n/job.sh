#!/bin/bash
# r06n (second call, timers made wave-uniform): config B's critical chain (first step).  Section profile of the timed kernel with
# -DCRT_PROFILE_PASS for (1) the first tile of the cost order only (the most expensive tile, whose wave lasts the
# whole launch on B) and (2) every wave, both on config B (1280x720, 256 spp, 20 bounces, seed 41).
# Prediction: the critical wave runs ~60k iterations at ~2.4k cycles each; its node steps and leaf rounds take a
# larger share than on the average wave, since few of its lanes park together.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06n; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
CRT_HIP_LIB=$LX/passcrit/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py --w 1280 --h 720 --spp 256 > $OUT/B_crit.json 2> $OUT/B_crit.err
CRT_HIP_LIB=$LX/pass/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py --w 1280 --h 720 --spp 256 > $OUT/B_all.json 2> $OUT/B_all.err
CRT_HIP_LIB=$LX/pass/libcrt_hip.so timeout -k 10 300 python3 -u tools/pass_profile.py > $OUT/C256_all.json 2> $OUT/C256_all.err
echo job done
