# Per-rank shares of the strong-scaled frame: the 2000-spp frame's spp/N on one GPU (N = 1, 2, 4, 8)
OUT=gpurun_out/r01aq
mkdir -p $OUT
set -e
for spp in 2000 1000 500 250; do
  timeout -k 10 300 python3 bench.py --spp $spp --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-count > $OUT/share_$spp.log 2>&1
done
for spp in 2000 1000 500 250; do echo "$spp $(grep -o '"ms_per_step": [0-9.]*\|"render_kernel_ms_avg": [0-9.]*\|"value": [0-9.]*' $OUT/share_$spp.log | tr '\n' ' ')"; done > $OUT/summary.txt
echo done
