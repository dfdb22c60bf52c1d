# variant 9 (K tiles per wave, lanes take the wave's pixels in turn) vs 8 at 2000 spp
OUT=gpurun_out/r01z
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k "persistent or xcd or first_block or tiles_per_wave" -v --timeout 240 --timeout-method thread > $OUT/pytest_order.log 2>&1
grep -q "failed" $OUT/pytest_order.log && { echo "order tests failed"; exit 1; }
set -e
timeout -k 10 700 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V8:o6,w4:l4:t2:T40:V9:o6:K2,w4:l4:t2:T40:V9:o6:K3,w4:l4:t2:T40:V9:o6:K4,w4:l4:t2:T40:V8:o6,w4:l4:t2:T40:V9:o6:K2" > $OUT/eval_v9_2000.log 2>&1
echo done
