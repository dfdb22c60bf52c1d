#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05d: pass / step micro-changes (a wave-uniform skip of a per-ray sphere no lane reaches, the wave's ray count by an
# LDS add without return, the leaf-span bounds check moved from every leaf step to the host's emission) against the
# previous commit (lib_exp/base): bit identity (tools/frame_hash.py), then interleaved main-kernel times on C, B and E.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05d; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
B="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/base/libcrt_hip.so > $OUT/sha.txt
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
done
for f in $OUT/*_[0-9].log; do echo "$(basename $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["render_phases_ms_avg"]["main_kernel_ms"], d["value"])')"; done | sort
echo job done
