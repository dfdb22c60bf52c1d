# r01j: GPU tests + smoke + bench with per-rank shading records, A/B against the HEAD build, rocprof
set -e
OUT=gpurun_out/r01j
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/head/libcrt_hip.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > $OUT/bench_head.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
echo done
