#!/bin/bash
# r06n (third call): config B's critical wave over time (tools/crit_trace.py, -DCRT_PROFILE_CRIT_TRACE
# -DCRT_PROFILE_WAVE_TIMES).  Prediction: early iterations (SIMD shared with 5 other waves) are 2-3x slower than the
# last ones (SIMD alone), so most of the chain is paced by sharing, not by its own latency.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06n; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
LX=$R/raytracer-cuda_amd/lib_exp
CRT_HIP_LIB=$LX/crit/libcrt_hip.so timeout -k 10 300 python3 -u tools/crit_trace.py > $OUT/B_crit_trace.json 2> $OUT/B_crit_trace.err
echo job done
