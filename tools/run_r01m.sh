# occupancy 6 without hot-path spills vs 5 (same box), 64 spp
set -e
OUT=gpurun_out/r01m
mkdir -p $OUT
timeout -k 10 300 python3 -m pytest tests/test_gpu_rebuilt.py -x -q > $OUT/pytest.log 2>&1
timeout -k 10 500 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4,w4:l4:t2:T40:V4:o6,w4:l4:t2:T36:V4:o6,w4:l4:t2:T44:V4:o6,w4:l4:t2:T40:V4" > $OUT/eval.log 2>&1
echo done
