# A/B/C on one box: prev = HEAD; pin = the link-row pin after the box tests (all seven node loads in flight
# together); new = pin + the shading record loaded before the per-ray sphere test
OUT=gpurun_out/r01ar
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py tests/test_gpu_primitives.py tests/test_gpu_bvh_build.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
E="python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs w4:l4:t2:T44:V8:o6"
for rep in 1 2; do
  CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/prev/libcrt_hip.so timeout -k 10 300 $E > $OUT/eval_prev_$rep.log 2>&1
  CRT_HIP_LIB=raytracer-cuda_amd/lib_exp/pin/libcrt_hip.so timeout -k 10 300 $E > $OUT/eval_pin_$rep.log 2>&1
  timeout -k 10 300 $E > $OUT/eval_new_$rep.log 2>&1
done
for f in $OUT/eval_*.log; do echo "$f $(grep -o '"kernel_ms": [0-9.]*' $f | tail -1) $(grep -o '"pixels_bit_equal": [0-9.]*' $f | tail -1)"; done > $OUT/summary.txt
echo done
