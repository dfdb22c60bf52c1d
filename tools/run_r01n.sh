# occupancy 6 default: GPU tests, smoke, bench + rocprof; occupancy 7 probe at 64 spp
set -e
OUT=gpurun_out/r01n
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V4:o7,w4:l4:t2:T40:V4:o5" > $OUT/eval_occ.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
echo done
