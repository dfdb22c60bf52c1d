# GPU round: tests, smoke, default bench, rocprofv3 kernel stats of the bench (each step bounded)
set -e
OUT=gpurun_out/${1:-check}
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
if [ -z "$SKIP_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
fi
echo done
