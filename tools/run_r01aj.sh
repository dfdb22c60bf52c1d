# A/B: leaf-round pair prefix folded into the LDS ray record (default lib) vs the previous commit (lib_exp/prev);
# regeneration threshold 40/44/48 on the new lib; rebuilt-path GPU tests
OUT=gpurun_out/r01aj
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py tests/test_gpu_primitives.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
for rep in 1 2; do
  CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/prev/libcrt_hip.so timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs w4:l4:t2:T44:V8:o6 > $OUT/eval_prev_$rep.log 2>&1
  timeout -k 10 400 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs w4:l4:t2:T44:V8:o6,w4:l4:t2:T40:V8:o6,w4:l4:t2:T48:V8:o6 > $OUT/eval_new_$rep.log 2>&1
done
for f in $OUT/eval_*.log; do echo "$f"; grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*' $f | paste - - ; done > $OUT/summary.txt
echo done
