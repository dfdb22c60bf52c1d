#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05ad: per-ray spheres after the trace: discriminants first, and a sphere no lane of the wave needs (no root, both
# roots behind, or beyond the hit) skips its reference box test (wave-uniform).  Prediction: frames identical; C -0.5 .. -1.5 %.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05ad; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_primitives.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_prim.log 2>&1
tail -1 $OUT/pytest_prim.log
B="CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
timeout -k 10 200 python3 -u tools/frame_hash.py --big > $OUT/hash_new.txt 2>&1
env $B timeout -k 10 200 python3 -u tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp $OUT/hash_new.txt $OUT/hash_base.txt && echo hashes identical
for i in 1 2; do
  env $B timeout -k 10 300 python3 -u tools/cold_ab.py --configs B,C,E --occupancy 0 --reps 1 > $OUT/base_$i.log 2>&1
  timeout -k 10 300 python3 -u tools/cold_ab.py --configs B,C,E --occupancy 0 --reps 1 > $OUT/new_$i.log 2>&1
done
grep -h '"rep": 1' $OUT/base_*.log $OUT/new_*.log | cut -c1-160
echo job done
