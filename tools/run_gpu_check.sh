# GPU round: tests, smoke, default bench (each step bounded; stop at the first failure)
set -e
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
echo done
