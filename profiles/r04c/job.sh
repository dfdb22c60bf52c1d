#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04c: (1) the wave's ray count in LDS instead of a VGPR (in-tree) against HEAD's build (base): bits + A/B;
# (2) carry mode 2 with round 0 peeled (no hot-loop spills): bits, the rebuilt-BVH GPU tests, section profile, sweep.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04c; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/*/libcrt_hip.so > $OUT/sha.txt
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
C2=$R/raytracer-cuda_amd/lib_exp/carry2/libcrt_hip.so
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$BASE timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
CRT_HIP_LIB=$C2 timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_carry2.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_base.txt) && echo "intree vs base: identical" || echo "intree vs base: DIFFER"
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt | cut -d' ' -f1-6) <(grep -v amdgpu.ids $OUT/hash_carry2.txt | cut -d' ' -f1-6) && echo "carry2 frames: identical" || echo "carry2 frames: DIFFER"
CRT_HIP_LIB=$C2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_rebuilt_carry2.log 2>&1 || echo "carry2 rebuilt tests: FAILED"
tail -1 $OUT/pytest_rebuilt_carry2.log
CRT_HIP_LIB=$C2 timeout -k 10 300 python3 tools/section_profile.py --spp 256 > $OUT/section_C256_carry2.txt 2>&1
timeout -k 10 300 python3 tools/section_profile.py --spp 256 > $OUT/section_C256.txt 2>&1
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  timeout -k 10 300 $B > $OUT/A_$i.log 2>&1
  CRT_HIP_LIB=$BASE timeout -k 10 300 $B > $OUT/base_$i.log 2>&1
  CRT_HIP_LIB=$C2 timeout -k 10 300 $B --carry 16 63 > $OUT/c2_16_63_$i.log 2>&1
  CRT_HIP_LIB=$C2 timeout -k 10 300 $B --carry 8 63 > $OUT/c2_8_63_$i.log 2>&1
  CRT_HIP_LIB=$C2 timeout -k 10 300 $B --carry 32 63 > $OUT/c2_32_63_$i.log 2>&1
  CRT_HIP_LIB=$C2 timeout -k 10 300 $B --carry 16 32 > $OUT/c2_16_32_$i.log 2>&1
  for f in A base c2_16_63 c2_8_63 c2_32_63 c2_16_32; do
    echo "$f round $i: $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"
  done
done
echo job done
