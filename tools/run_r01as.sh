# A/B: 4-wide slab test as one packed FMA per plane pair (lo * inv - o * inv) vs (lo - o) * inv (lib_exp/prev = HEAD);
# per-ray agreement with the reference BVH on config C (crt_scene_compare) and config E, then interleaved timing
OUT=gpurun_out/r01as
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py tests/test_gpu_primitives.py tests/test_gpu_bvh_build.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python3 tools/bvh_eval.py --spp 32 --reps 1 --configs w4:l4:t2:T44:V8:o6 > $OUT/compare_C.log 2>&1
timeout -k 10 300 python3 tools/bvh_eval.py --scene cornell_1m --spp 16 --reps 1 --configs w4:l4:t2:T44:V8:o6 > $OUT/compare_E.log 2>&1
E="python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs w4:l4:t2:T44:V8:o6"
for rep in 1 2; do
  CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/prev/libcrt_hip.so timeout -k 10 300 $E > $OUT/eval_prev_$rep.log 2>&1
  timeout -k 10 300 $E > $OUT/eval_new_$rep.log 2>&1
done
for f in $OUT/eval_*.log $OUT/compare_*.log; do echo "$f $(grep -o '"kernel_ms": [0-9.]*' $f | tail -1) $(grep -o '"pixels_bit_equal": [0-9.]*' $f | tail -1) $(grep -o '"per_ray": {[^}]*}' $f | tail -1)"; done > $OUT/summary.txt
echo done
