# r03e: the sharded multi-rank path with the HIP kernel (gloo, ranks sharing cuda:0)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1
tail -5 $OUT/pytest_dist.log
