# re-entry check of the restored tree: GPU tests, smoke, bench, rocprofv3 kernel stats, PMC HBM traffic
# of the default (occupancy-6) kernel
set -e
OUT=gpurun_out/r01o
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
cd $R
SKIP_SQ=1 bash tools/pmc.sh $OUT/pmc
echo done
