# r03s: variant 10 (variant 3's program, tiled one-wave workgroups + probe order) on the reference BVH
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03s; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_checked.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -2 $OUT/pytest.log
B="python3 bench.py --no-cpu-baseline --no-count --no-parity --bvh reference"
for i in 1 2; do
  timeout -k 10 300 $B --kernel-variant 3 > $OUT/C_v3_$i.log 2>&1
  timeout -k 10 300 $B --kernel-variant 10 > $OUT/C_v10_$i.log 2>&1
done
for f in $OUT/C_*.log; do echo "$(basename $f) $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f) $(grep -o '"render_phases_ms_last_frame": {[^}]*}' $f)"; done
