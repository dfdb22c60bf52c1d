#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04u: config B's occupancy (6, the automatic choice below 4 tiles per wave slot, against 7) with the wave drain on.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04u; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 tools/schedule_sweep.py --world 1 --width 1280 --height 720 --spp 256 --reps 5 --set auto: occ7:occ=7 occ6:occ=6 > $OUT/sweep_B.jsonl
python3 -c "
import json
for d in map(json.loads, open('$OUT/sweep_B.jsonl')): print(d['name'], d['main_median_ms'], d['main_ms_reps'], d['kernel'])"
echo job done
