#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05y: helper lanes (variant 8, CRT_HELPER_TILES): idle lanes of a step test a node from a tracing lane's stack.
# Predictions: frames/RNG/rays identical at every setting; B (few tiles per slot, chain-bound) -5 .. -15 % with helpers
# on all tiles or the first 1024; C +0 .. +2 % at 0 against the base library (more spills), -3 .. +5 % with helpers on.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05y; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u tools/help_ab.py --parity --configs B --values 0,-1,1024 --reps 3 > $OUT/help_B.log 2>&1
grep -v '"rep": 0' $OUT/help_B.log | cut -c1-250
CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_host.so \
  timeout -k 10 300 python3 -u tools/help_ab.py --configs B --values 0 --reps 3 > $OUT/base_B.log 2>&1
grep -v '"rep": 0' $OUT/base_B.log | cut -c1-200
timeout -k 10 400 python3 -u tools/help_ab.py --configs C --values 0,-1 --reps 2 > $OUT/help_C.log 2>&1
grep -v '"rep": 0' $OUT/help_C.log | cut -c1-200
CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_host.so \
  timeout -k 10 300 python3 -u tools/help_ab.py --configs C --values 0 --reps 2 > $OUT/base_C.log 2>&1
grep -v '"rep": 0' $OUT/base_C.log | cut -c1-200
echo job done
