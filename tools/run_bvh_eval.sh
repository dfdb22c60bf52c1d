set -e
mkdir -p gpurun_out/bvh3
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > gpurun_out/bvh3/pytest_gpu.log 2>&1
timeout -k 10 500 python3 tools/bvh_eval.py --configs "w4:l4:t1,w4:l4:t1:o4,w4:l8:t2,w4:l4:t3,w2:l16:t6" > gpurun_out/bvh3/eval.log 2>&1
echo done
