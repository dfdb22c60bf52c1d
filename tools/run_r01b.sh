set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r01b
timeout -k 10 400 python3 bench.py > gpurun_out/r01b/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01b/prof -o bench -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r01b/bench_prof.log 2>&1
echo done
