# r03n: depth-first vs breadth-first emission of the 4-wide nodes (CRT_WIDE_ORDER=dfs), configs C and E, interleaved
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03n; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  timeout -k 10 300 $B > $OUT/C_bfs_$i.log 2>&1
  CRT_WIDE_ORDER=dfs timeout -k 10 300 $B > $OUT/C_dfs_$i.log 2>&1
  timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E_bfs_$i.log 2>&1
  CRT_WIDE_ORDER=dfs timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E_dfs_$i.log 2>&1
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"render_kernel_ms_avg": [0-9.]*' $f)"; done
