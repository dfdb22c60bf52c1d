set -e
mkdir -p gpurun_out/occ6
timeout -k 10 300 python3 -m pytest tests/test_gpu_rebuilt.py -x -q > gpurun_out/occ6/pytest.log 2>&1
timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t3:T40,w4:l4:t3:T40:o6,w4:l4:t3:T48:o6,w4:l4:t3:T32:o6,w4:l8:t3:T40:o6" > gpurun_out/occ6/eval.log 2>&1
echo done
