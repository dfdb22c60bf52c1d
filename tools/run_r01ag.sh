# A/B: merged scatter draw + per-ray spheres after the trace (default lib) vs spheres first (lib_exp/sfirst)
# vs the previous commit (lib_exp/head); correctness of the default lib on the rebuilt/primitive/parity suites
OUT=gpurun_out/r01ag
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py tests/test_gpu_primitives.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
C="w4:l4:t2:T44:V8:o6"
for rep in 1 2; do
  for lib in head new sfirst; do
    if [ $lib = new ]; then L=""; else L=raytracer-cuda_amd/lib_exp/$lib/libcrt_hip.so; fi
    CRT_HIP_LIB=$L timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs $C > $OUT/eval_${lib}_$rep.log 2>&1
    echo "$lib $rep $(grep -o '"kernel_ms": [0-9.]*' $OUT/eval_${lib}_$rep.log | tail -1)" | tee -a $OUT/summary.txt
  done
done
echo done
