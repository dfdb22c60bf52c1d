# Variant 6 (deferred leaf rounds) vs variant 4: parity tests, 64-spp timing + section profile; per-ray sphere cost
set -e
OUT=gpurun_out/defer
mkdir -p $OUT
timeout -k 10 300 python3 -m pytest tests/test_gpu_rebuilt.py -x -q > $OUT/pytest.log 2>&1
timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4,w4:l4:t2:T40:V6,w4:l4:t2:T32:V6,w4:l4:t2:T48:V6,w4:l8:t2:T40:V6,w4:l3:t2:T40:V6" > $OUT/eval.log 2>&1
CRT_HIP_LIB=$GRAFT_REPO_ROOT/raytracer-cuda_amd/lib_exp/nosph/libcrt_hip.so timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4" > $OUT/eval_nosph.log 2>&1
echo done
