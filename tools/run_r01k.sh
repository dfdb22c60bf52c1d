# exact fast reciprocal in unit() / roulette / ior: full GPU tests; 64-spp timing vs HEAD build; L1 node-prefetch probe;
# exhaustive v_sqrt_f32 rounding probe
set -e
OUT=gpurun_out/r01k
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 120 ./tools/probes/sqrt_probe > $OUT/sqrt_probe.log 2>&1
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4" > $OUT/eval_new.log 2>&1
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/head/libcrt_hip.so timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4" > $OUT/eval_head.log 2>&1
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/pf/libcrt_hip.so timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4" > $OUT/eval_pf.log 2>&1
echo done
