# Sweep at HEAD: regeneration threshold T 40..52 at occupancy 6, and occupancy 7 at T44 (variant 8, 2000 spp)
OUT=gpurun_out/r01ap
mkdir -p $OUT
set -e
timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 2 --configs w4:l4:t2:T44:V8:o6,w4:l4:t2:T40:V8:o6,w4:l4:t2:T48:V8:o6,w4:l4:t2:T52:V8:o6,w4:l4:t2:T44:V8:o7,w4:l4:t2:T44:V8:o6 > $OUT/sweep.log 2>&1
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*\|"pixels_bit_equal": [0-9.]*' $OUT/sweep.log | paste - - - > $OUT/summary.txt || true
echo done
