# r03b: A/B of the leaf-round atomic sinks (CRT_LEAF_DUMMY) and the SBVH tree on configs C and E
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03b; mkdir -p $OUT
bash tools/gpu_job.sh ab r03b/ab_leaf raytracer-cuda_amd/lib_exp/leafdummy/libcrt_hip.so 3
for f in $OUT/ab_leaf/*.log; do echo "$f $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f)"; done
for i in 1 2; do
  for v in base sbvh; do
    a=""; [ $v = sbvh ] && a="--spatial-splits"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --steps 2 $a > $OUT/C_${v}_$i.log 2>&1
    echo "C $v $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/C_${v}_$i.log) $(grep -o '"per_ray": {[^}]*}' $OUT/C_${v}_$i.log)"
  done
done
for i in 1 2; do
  for v in base sbvh; do
    a=""; [ $v = sbvh ] && a="--spatial-splits"
    timeout -k 10 300 python3 bench.py --scene cornell_1m --spp 512 --no-cpu-baseline --no-parity --steps 2 $a > $OUT/E_${v}_$i.log 2>&1
    echo "E $v $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/E_${v}_$i.log) $(grep -o '"per_ray": {[^}]*}' $OUT/E_${v}_$i.log)"
  done
done
