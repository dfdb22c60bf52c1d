# r03c: the GPU suite at the working tree (checked build, SBVH configs, variant 8 vs oracle), then the leaf-round
# self-slot atomics A/B (CRT_LEAF_SELF)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
bash tools/gpu_job.sh ab r03c/ab_self raytracer-cuda_amd/lib_exp/leafself/libcrt_hip.so 3
for f in $OUT/ab_self/*.log; do echo "$f $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f)"; done
# the box's CPU allocation (for bench.py's cpu_baseline legs)
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS";
  python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; grep -m1 "model name" /proc/cpuinfo; } > $OUT/cpu_share.txt 2>&1
cat $OUT/cpu_share.txt
