#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05e: (1) r05d measured the three micro-changes together at C +0.45 %, B -1.3 %, E +0.4 %: bisect them on C and B,
# each alone on top of e93226f (lib_exp/m_*: base, sphere = the per-sphere wave-uniform skip, span = the leaf-span check
# on the host, lds = the ray count by an LDS add), 3 interleaved rounds.
# (2) the live-lane time histogram (lib_exp/live): how much wave time the drain takes, i.e. the ceiling of (3).
# (3) variant 11 (variant 8 + straggler consolidation, in-tree library): bit identity, then main-kernel times on B, the
# N = 8 share and C.  Predicted: a gain of at most the wave-time share spent at <= 8-16 live lanes, minus the consumers'
# own cost; a loss if consumers' full waves slow the stragglers' chains at the end of the launch.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05e; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/*/libcrt_hip.so > $OUT/sha.txt
BN="--no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  for n in base sphere span lds; do
    L="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/m_$n/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/m_$n/libcrt_host.so"
    env $L timeout -k 10 300 python3 bench.py $BN > $OUT/C_${n}_$i.log 2>&1
    env $L timeout -k 10 300 python3 bench.py $BN --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_${n}_$i.log 2>&1
  done
done
for f in $OUT/*_[0-9].log; do echo "$(basename $f) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["render_phases_ms_avg"]["main_kernel_ms"], d["value"])')"; done | sort
LV="CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/live/libcrt_hip.so"
env $LV timeout -k 10 120 python3 tools/live_histogram.py --spp 2000 > $OUT/live_C.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --spp 250 > $OUT/live_N8.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --w 1280 --h 720 --spp 256 > $OUT/live_B.json 2>&1
env $LV timeout -k 10 120 python3 tools/live_histogram.py --scene cornell_1m --spp 512 > $OUT/live_E.json 2>&1
tail -qn1 $OUT/live_*.json
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
