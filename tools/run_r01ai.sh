# occupancy 7 vs 6 for variant 8 after the shading-pass cuts (one box, interleaved)
OUT=gpurun_out/r01ai
mkdir -p $OUT
set -e
timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T44:V8:o6,w4:l4:t2:T44:V8:o7,w4:l4:t2:T44:V8:o6,w4:l4:t2:T44:V8:o7" > $OUT/eval_occ.log 2>&1
grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*' $OUT/eval_occ.log | paste - - > $OUT/summary.txt
echo done
