#!/bin/bash
# r06z8: the launch's tail rendered in half tiles (experiment -DCRT_TAIL_SPLIT_EXP; CRT_TAIL_SPLIT=K: the last K tiles
# of the cost order as two workgroups of 4 rows each, lanes 32-63 idle), so the drain ends on finer-grained waves.
# Frame hashes with K = 0 and K = 64 (every case of tools/frame_hash.py --big), then config C main kernel at K = 0, 2048,
# 7168, 14336, two rounds; and the N = 8 share at K = 0 and 7168.  Prediction: bit-identical; C -0.5 to -2 % at the best
# K (the drain costs ~6 % of the slot-time, r04j), worse at the largest K (half-empty waves are half as efficient).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z8; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
L=$R/raytracer-cuda_amd/lib_exp/tail/libcrt_hip.so
CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$L timeout -k 10 300 python3 -u tools/frame_hash.py --big > $OUT/hash_k0.txt 2> $OUT/hash.err
CRT_TAIL_SPLIT=64 CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$L timeout -k 10 300 python3 -u tools/frame_hash.py --big > $OUT/hash_k64.txt 2>> $OUT/hash.err
B="python3 bench.py --no-cpu-baseline --no-count --no-parity --steps 3 --warmup 1"
for rep in 1 2; do
  for k in 0 2048 7168 14336; do
    CRT_TAIL_SPLIT=$k CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$L timeout -k 10 300 $B > $OUT/C_k${k}_$rep.log 2>&1
  done
  for k in 0 7168; do
    CRT_TAIL_SPLIT=$k CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$L timeout -k 10 300 $B --share 0 8 > $OUT/S8_k${k}_$rep.log 2>&1
  done
done
echo job done
