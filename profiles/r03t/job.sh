# r03t: the GPU suite with variant 10 as the automatic choice for threaded scenes; default bench
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | grep -o '"value": [0-9.]*\|"parity": {[^}]*}'
