# full GPU suite after the RNG cache / automatic probe / tile key defaults; bench; regen-threshold repeat
OUT=gpurun_out/r01af
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
timeout -k 10 900 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V8:o6,w4:l4:t2:T44:V8:o6,w4:l4:t2:T48:V8:o6,w4:l4:t2:T40:V8:o6,w4:l4:t2:T44:V8:o6,w4:l4:t2:T48:V8:o6" > $OUT/eval_T_2000.log 2>&1
echo done
