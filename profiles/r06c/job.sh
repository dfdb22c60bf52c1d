#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06c: (1) VERDICT r5 item 2's prediction: the rejection loops counted per wave in the profiling build
# (CRT_PROFILE_LOOPS) at 256 spp on config C's frame and at 2000 spp; prediction: a fused loop saves at most 1-2 % of
# the kernel's VALU.  (2) The N = 8 share line with its own counters: bench.py --share 0 8.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06c; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/loops/libcrt_hip.so timeout -k 10 300 python3 tools/loop_fusion_count.py --spp 256 > $OUT/loops_C256.json 2> $OUT/loops_C256.err
CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/loops/libcrt_hip.so timeout -k 10 300 python3 tools/loop_fusion_count.py --spp 2000 > $OUT/loops_C2000.json 2> $OUT/loops_C2000.err
timeout -k 10 300 python3 bench.py --share 0 8 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_share8.log 2>&1
echo job done
