# the per-GPU share at N=8 (250 spp) and N=4 (500 spp): probe spp and variant choice
OUT=gpurun_out/r01ad
mkdir -p $OUT
set -e
timeout -k 10 500 python3 tools/bvh_eval.py --no-compare --spp 250 --reps 2 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P4,w4:l4:t2:T40:V8:o6:P2,w4:l4:t2:T40:V8:o6:P1,w4:l4:t2:T40:V8:o6:P0,w4:l4:t2:T40:V7:o6:P0" > $OUT/eval_250.log 2>&1
timeout -k 10 500 python3 tools/bvh_eval.py --no-compare --spp 500 --reps 1 --configs "w4:l4:t2:T40:V8:o6:P4,w4:l4:t2:T40:V8:o6:P2" > $OUT/eval_500.log 2>&1
echo done
