#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05d: (1) pass / step micro-changes (a wave-uniform skip of a per-ray sphere no lane reaches, the wave's ray count by an
# LDS add without return, the leaf-span bounds check moved from every leaf step to the host's emission) against the
# previous commit (lib_exp/base): bit identity (tools/frame_hash.py), then interleaved main-kernel times on C, B and E.
# Predicted: C -1 to -1.5 % (the metal sphere's quadratic skipped in most passes: ~25 of ~640 pass VALU; the leaf step
# loses a kernel-argument reload, its wait and ~5 VALU).  Then the live-lane time histogram (lib_exp/live,
# -DCRT_PROFILE_LIVE): how much wave time is spent with few live lanes, the ceiling of any straggler consolidation.
# (2) variant 11 = variant 8 + straggler consolidation (in-tree library): bit identity and main-kernel times on B, the
# N = 8 share and C.  Predicted: the share of wave time spent at <= 8 live lanes (from the histogram) minus the consumer
# waves' own cost; a loss if the consumers' full waves slow the stragglers' sample chains at the end of the launch.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05d; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
A="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/microA/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/microA/libcrt_host.so"
B="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
sha256sum raytracer-cuda_amd/lib_exp/microA/libcrt_hip.so raytracer-cuda_amd/lib_exp/base/libcrt_hip.so > $OUT/sha.txt
env $A timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_A.txt 2>&1
env $B timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp $OUT/hash_A.txt $OUT/hash_base.txt && echo "hashes identical" | tee $OUT/hash_cmp.txt
BN="--no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  env $A timeout -k 10 300 python3 bench.py $BN > $OUT/C_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN > $OUT/C_base_$i.log 2>&1
  env $A timeout -k 10 300 python3 bench.py $BN --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_base_$i.log 2>&1
  env $A timeout -k 10 300 python3 bench.py $BN --scene cornell_1m --spp 512 > $OUT/E_A_$i.log 2>&1
  env $B timeout -k 10 300 python3 bench.py $BN --scene cornell_1m --spp 512 > $OUT/E_base_$i.log 2>&1
done
LV="CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/live/libcrt_hip.so"
env $LV timeout -k 10 120 python3 tools/live_histogram.py --spp 2000 > $OUT/live_C.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --spp 250 > $OUT/live_N8.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --w 1280 --h 720 --spp 256 > $OUT/live_B.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --scene cornell_1m --spp 512 > $OUT/live_E.json 2>&1
tail -qn1 $OUT/live_*.json
for f in $OUT/*_[0-9].log; do echo "$(basename $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["render_phases_ms_avg"]["main_kernel_ms"], d["value"])')"; done | sort
# variant 11 (straggler consolidation): bit identity, then variant 8 vs 11 at hand-off lanes 4/8/16 interleaved
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "consolidation or wave_drain" > $OUT/pytest_v11.log 2>&1
S="v8:v=8 c8:v=11,cl=8 c16:v=11,cl=16 c8e0:v=11,cl=8,ce=0 c8e5:v=11,cl=8,ce=5,cm=16 c16t16:v=11,cl=16,ct=16"
timeout -k 10 300 python3 tools/schedule_sweep.py --width 1280 --height 720 --spp 256 --world 1 --reps 3 --set $S > $OUT/v11_B.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 3 --set $S > $OUT/v11_N8.jsonl
timeout -k 10 600 python3 tools/schedule_sweep.py --world 1 --reps 2 --set $S > $OUT/v11_C.jsonl
for f in B N8 C; do python3 -c "
import json
for d in map(json.loads, open('$OUT/v11_$f.jsonl')): print('$f', d['name'], d['main_median_ms'], d['main_ms_reps'], d.get('rays'), d.get('cons'))"; done
echo job done
