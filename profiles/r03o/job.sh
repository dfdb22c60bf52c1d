# r03o: SAH bin count 32 (in-tree) / 64 / 128, configs C and E, 3 interleaved rounds (confirmation of r02az)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03o; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  for b in 32 64 128; do
    L=""; [ $b != 32 ] && L=$R/raytracer-cuda_amd/lib_exp/b$b/libcrt_hip.so
    CRT_HIP_LIB=$L timeout -k 10 300 $B > $OUT/C_b${b}_$i.log 2>&1
    CRT_HIP_LIB=$L timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E_b${b}_$i.log 2>&1
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f)"; done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1
tail -2 $OUT/pytest_dist.log
