# r03g: variant 7 with a refill threshold vs variant 8, configs C and B
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03g; mkdir -p $OUT
timeout -k 10 400 python3 tools/refill_sweep.py --refill 64,32,16,8,4 --reps 2 > $OUT/sweep_C.log 2>&1
tail -1 $OUT/sweep_C.log
timeout -k 10 200 python3 tools/refill_sweep.py --w 1280 --h 720 --spp 256 --refill 32,16,8 --reps 3 > $OUT/sweep_B.log 2>&1
tail -1 $OUT/sweep_B.log
