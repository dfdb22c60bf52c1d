#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06g: the pass's "rest" (10 % of the timed kernel's wave cycles at C, r06f) ends in the variant-8 ray count, an LDS
# read-modify-write by lane 0 behind an `s_waitcnt vmcnt(0)` (the register it reads into may be the data of a pending
# overflow-stack store).  -DCRT_RAYS_SGPR keeps the wave's ray count in an SGPR instead (compile: 72 VGPRs, 3 VGPR
# spills as before, 19 SGPR spills (+2); cost-model screen "open").  Prediction: C -0.5 .. -2 %, B similar; frames
# identical.  Then the timed-kernel pass profile of the variant.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06g; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
V=raytracer-cuda_amd/lib_exp/rsgpr/libcrt_hip.so
timeout -k 10 300 python3 tools/frame_hash.py > $OUT/hash_A.txt 2>&1
CRT_HIP_LIB=$R/$V timeout -k 10 300 python3 tools/frame_hash.py > $OUT/hash_B.txt 2>&1
cmp $OUT/hash_A.txt $OUT/hash_B.txt && echo "hashes identical" > $OUT/hash_cmp.txt
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity > $OUT/C_A_$i.log 2>&1
  CRT_HIP_LIB=$R/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity > $OUT/C_B_$i.log 2>&1
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity --width 1280 --height 720 --spp 256 --steps 8 > $OUT/B_A_$i.log 2>&1
  CRT_HIP_LIB=$R/$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity --width 1280 --height 720 --spp 256 --steps 8 > $OUT/B_B_$i.log 2>&1
done
for f in $OUT/C_*_*.log $OUT/B_*_*.log; do echo "$(basename $f): $(grep -o '"main_kernel_ms": [0-9.]*' $f | tail -1)"; done > $OUT/summary.txt
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/passr/libcrt_hip.so timeout -k 10 300 python3 tools/pass_profile.py --spp 256 > $OUT/pass_C256_rsgpr.json 2>/dev/null
echo job done
