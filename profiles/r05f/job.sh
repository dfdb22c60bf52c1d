#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05f: variant 11 again after r05e's fault (a consumer read `taken` after `reserved`, so a concurrent claim could make
# its window underflow and claim entries never written; fixed: taken is read first, a never-written entry leaves the lane
# idle and counts a spin-out).  Variant 11 (variant 8 + straggler consolidation, in-tree library): bit identity, then main-kernel times on B, the
# N = 8 share and C.  Predicted: a gain of at most the wave-time share spent at <= 8-16 live lanes, minus the consumers'
# own cost; a loss if consumers' full waves slow the stragglers' chains at the end of the launch.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05f; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
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
