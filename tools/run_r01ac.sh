# variant 8 tile keys (slowest pixel / + mean / neighbourhood-raised) at 2000 spp
OUT=gpurun_out/r01ac
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k "persistent or xcd or first_block or tiles_per_wave or key" -v --timeout 240 --timeout-method thread > $OUT/pytest_order.log 2>&1
grep -q "failed" $OUT/pytest_order.log && { echo "order tests failed"; exit 1; }
set -e
timeout -k 10 700 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V8:o6,w4:l4:t2:T40:V8:o6:Y1,w4:l4:t2:T40:V8:o6:Y2,w4:l4:t2:T40:V8:o6,w4:l4:t2:T40:V8:o6:Y1,w4:l4:t2:T40:V8:o6:Y2" > $OUT/eval_keys_2000.log 2>&1
echo done
