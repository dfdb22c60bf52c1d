# Configs B and E at HEAD through bench.py (N = 1, with the reference-BVH parity frame), config C at 250 spp
# (rank 0's share at N = 8)
OUT=gpurun_out/r01av
mkdir -p $OUT
set -e
timeout -k 10 400 python3 bench.py --width 1280 --height 720 --spp 256 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_B.log 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_E.log 2>&1
timeout -k 10 300 python3 bench.py --spp 250 --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-count > $OUT/share_250.log 2>&1
echo done
