# r03r: 256 SAH bins and 128-bin SBVH against the 128-bin default, configs C and E, 3 interleaved rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03r; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
L256=$R/raytracer-cuda_amd/lib_exp/b256/libcrt_hip.so
for i in 1 2 3; do
  for s in C E; do
    A=""; [ $s = E ] && A="--scene cornell_1m --spp 512"
    timeout -k 10 300 $B $A > $OUT/${s}_b128_$i.log 2>&1
    CRT_HIP_LIB=$L256 timeout -k 10 300 $B $A > $OUT/${s}_b256_$i.log 2>&1
    timeout -k 10 300 $B $A --spatial-splits > $OUT/${s}_sbvh128_$i.log 2>&1
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f) $(grep -o '"load_build_upload_s": [0-9.]*' $f)"; done
