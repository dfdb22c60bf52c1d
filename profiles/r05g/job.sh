#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05g: the camera re-read from the kernel arguments where next_ray needs it (in-tree) against HEAD (lib_exp/base).
# Kept in SGPRs across the loop the camera made the benchmarked kernel spill 17 SGPRs (26 v_readlane read-backs, three
# per stack push or pop) and reload other kernel arguments inside the loop; with the reload: 4 spilled SGPRs, 33 fewer
# static VALU.  Predicted: C -0.5 to -1.5 %, B and E similar or better, the 1-spp frame (variant 7: 22 -> 15 spills) better.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05g; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
B="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
sha256sum raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/base/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_A.txt 2>&1
env $B timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp $OUT/hash_A.txt $OUT/hash_base.txt && echo "hashes identical" | tee $OUT/hash_cmp.txt
BN="--no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py $BN > $OUT/C_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN > $OUT/C_base_$i.log 2>&1
  timeout -k 10 300 python3 bench.py $BN --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_base_$i.log 2>&1
  timeout -k 10 300 python3 bench.py $BN --scene cornell_1m --spp 512 > $OUT/E_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN --scene cornell_1m --spp 512 > $OUT/E_base_$i.log 2>&1
  timeout -k 10 300 python3 bench.py $BN --spp 1 --steps 50 --warmup 5 > $OUT/S1_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN --spp 1 --steps 50 --warmup 5 > $OUT/S1_base_$i.log 2>&1
done
for f in $OUT/*_[0-9].log; do echo "$(basename $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["render_phases_ms_avg"]["main_kernel_ms"], d["value"])')"; done | sort
echo job done
