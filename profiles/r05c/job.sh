#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05c: variant 8's tail mode (crt_renderer_set_tail_mode): bit-identity tests, then tail lanes 0/2/4/8/16 interleaved
# on config B (1280x720, 256 spp), config C (2000 spp) and the N = 8 rank share (250 spp).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05c; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rebuilt.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "tail_mode or wave_drain or persistent_queue or shipped" > $OUT/pytest_tail.log 2>&1
S="t0:tail=0 t2:tail=2 t4:tail=4 t8:tail=8 t16:tail=16"
timeout -k 10 300 python3 tools/schedule_sweep.py --width 1280 --height 720 --spp 256 --world 1 --reps 4 --set $S > $OUT/sweep_B.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 4 --set $S > $OUT/sweep_N8.jsonl
timeout -k 10 600 python3 tools/schedule_sweep.py --world 1 --reps 3 --set t0:tail=0 t4:tail=4 t8:tail=8 > $OUT/sweep_C.jsonl
for f in B N8 C; do python3 -c "
import json
for d in map(json.loads, open('$OUT/sweep_$f.jsonl')): print('$f', d['name'], d['main_median_ms'], d['main_ms_reps'], d.get('rays'))"; done
echo job done
