set -e
O=gpurun_out/dpp2
mkdir -p $O
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1
timeout -k 10 500 python3 tools/mismatch_dump.py $O > $O/log 2>&1
timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t3:T40" > $O/eval.log 2>&1
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench_C.log 2>&1
echo done
