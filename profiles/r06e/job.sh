#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06e: why the capped unit-sphere loop lost (r06d: bit-identical at caps 2/3/4, C +8.8 / +1.9 / +0.6 %).  Section
# profile of the counting kernel (s_memtime per section) at cap 0 / 3 / 2, and the loop counts of the profiling build
# (passes, loop maxima) at the same caps.  Expectation: the pass share falls and the traversal share rises (deferred
# lanes idle through the steps), passes per ray up ~10 % at cap 3.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06e; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
for cap in 0 3 2; do
  timeout -k 10 300 python3 tools/section_profile.py --spp 256 --sphere-cap $cap > $OUT/section_cap$cap.txt 2>&1
  CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/loops/libcrt_hip.so timeout -k 10 300 python3 tools/loop_fusion_count.py --spp 256 --sphere-cap $cap > $OUT/loops_cap$cap.json 2>/dev/null
done
echo job done
