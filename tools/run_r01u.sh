# work order experiments at the headline size: variant 4 vs 8 (row order, XCD bands, probe LPT, banded probe LPT)
OUT=gpurun_out/r01u
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k "persistent or xcd" -v --timeout 240 --timeout-method thread > $OUT/pytest_order.log 2>&1
grep -q "failed" $OUT/pytest_order.log && { echo "order tests failed"; exit 1; }
set -e
timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P0,w4:l4:t2:T40:V8:o6:P0:X1,w4:l4:t2:T40:V8:o6:P4,w4:l4:t2:T40:V8:o6:P4:X1,w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P0:X1" > $OUT/eval_order_2000.log 2>&1
echo done
