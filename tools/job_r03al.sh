#!/bin/bash
# r03al: occupancy chosen by tiles per wave slot (7 for config C/E-sized frames, 6 for config B): GPU suite, hashes,
# default bench (C), config B and E.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03al; OUT=$R/gpurun_out/$O; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
grep -v amdgpu.ids $OUT/hash_intree.txt
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
timeout -k 10 300 $B > $OUT/C.log 2>&1
timeout -k 10 300 $B --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B.log 2>&1
timeout -k 10 300 $B --scene cornell_1m --spp 512 > $OUT/E.log 2>&1
for f in C B E; do echo "$f: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $OUT/$f.log) $(grep -o '"value": [0-9.]*' $OUT/$f.log)"; done
