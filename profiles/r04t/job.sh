#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04t: variant 8's wave timelines at 250 and 2000 spp with the wave drain (48/64, the default) and without it (64/64):
# where the N = 8 rank share's time goes at the round-4 HEAD.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04t; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
WT=$R/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip $WT > $OUT/sha.txt
for spp in 250 2000; do
  for wd in 48 64; do
    CRT_HIP_LIB=$WT timeout -k 10 150 python3 tools/wave_timeline.py --variant 8 --spp $spp --wave-drain $wd >> $OUT/timeline_v8.jsonl 2>> $OUT/timeline.err
  done
done
python3 -c "
import json
for l in open('$OUT/timeline_v8.jsonl'):
    d=json.loads(l); print(d['spp'], d['wave_drain'], d['kernel_ms'], d['span_ms'], d['occupancy_efficiency'], d['tail_fraction'], d['wave_ms'], d['order']['model_span_ms_true_lpt'])"
echo job done
