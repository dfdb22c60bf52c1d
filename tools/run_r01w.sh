# variant 8 with a work-weighted probe (counting kernel) at 2, 4, 8 spp vs variant 4 at 2000 spp; 1-spp sweep
OUT=gpurun_out/r01w
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k "persistent or xcd or first_block" -v --timeout 240 --timeout-method thread > $OUT/pytest_order.log 2>&1
grep -q "failed" $OUT/pytest_order.log && { echo "order tests failed"; exit 1; }
set -e
timeout -k 10 700 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P4,w4:l4:t2:T40:V8:o6:P8,w4:l4:t2:T40:V8:o6:P2,w4:l4:t2:T40:V8:o6:P16,w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P8" > $OUT/eval_probe_2000.log 2>&1
timeout -k 10 300 python3 tools/variant_sweep.py --spps 1,4,16 > $OUT/sweep_low_spp.log 2>&1
echo done
