#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04x: the wave drain's fraction and the regeneration threshold around their defaults on config C itself (2000 spp),
# interleaved, for the next round's plan; no change to the tree.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04x; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 400 python3 tools/schedule_sweep.py --world 1 --reps 4 --set wd48: wd40:wd=40 wd56:wd=56 wd32:wd=32 wd64:wd=64 T42:T=42 T46:T=46 > $OUT/sweep_C.jsonl
python3 -c "
import json
for d in map(json.loads, open('$OUT/sweep_C.jsonl')): print(d['name'], d['main_median_ms'], d['main_ms_reps'])"
echo job done
