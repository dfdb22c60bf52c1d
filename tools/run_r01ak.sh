# variant 8 with pixel order (tile key 3: pixels by probe cost; 4: by 3x3-mean cost) vs tiles (key 2)
OUT=gpurun_out/r01ak
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py -x -q -k "key_modes or persistent_queue_variant" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
for rep in 1 2; do
  timeout -k 10 600 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs w4:l4:t2:T44:V8:o6:Y2,w4:l4:t2:T44:V8:o6:Y3,w4:l4:t2:T44:V8:o6:Y4 > $OUT/eval_$rep.log 2>&1
done
for f in $OUT/eval_*.log; do echo "$f"; grep -o '"config": "[^"]*"\|"kernel_ms": [0-9.]*' $f | paste - - ; done > $OUT/summary.txt
echo done
