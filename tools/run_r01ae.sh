# variant 8 parameter sweep at 2000 spp: occupancy, leaf size / SAH traversal cost, regen threshold
OUT=gpurun_out/r01ae
mkdir -p $OUT
set -e
timeout -k 10 900 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V8:o6,w4:l4:t2:T40:V8:o7,w4:l4:t2:T40:V8:o5,w4:l4:t3:T40:V8:o6,w4:l8:t2:T40:V8:o6,w4:l3:t2:T40:V8:o6,w4:l4:t1.5:T40:V8:o6,w4:l4:t2:T36:V8:o6,w4:l4:t2:T44:V8:o6,w4:l4:t2:T40:V8:o6" > $OUT/eval_sweep_2000.log 2>&1
echo done
