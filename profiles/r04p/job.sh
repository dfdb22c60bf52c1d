#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04p: two follow-ups of the wave drain. (1) The same rule for variant 7's persistent waves
# (profiles/r04p/v7_wave_drain.patch, built as lib_exp/v7wd, not in the tree): bits, the interactive loop and config A.
# (2) The regeneration threshold re-swept with the wave drain on (C, B and the N = 8 share).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04p; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
E=$R/raytracer-cuda_amd/lib_exp
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so $E/v7wd/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$E/v7wd/libcrt_hip.so CRT_HOST_LIB=$E/v7wd/libcrt_host.so timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_v7wd.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_v7wd.txt) && echo "v7wd identical" || echo "v7wd DIFFERS"
F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
for i in 1 2 3; do
  for v in intree v7wd; do
    if [ $v = v7wd ]; then L="LD_LIBRARY_PATH=$E/v7wd"; else L="X=1"; fi
    for s in still orbit; do
      env $L timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script $s -bvh rebuilt $F > $OUT/viewer_${s}_${v}_$i.json
    done
    if [ $v = v7wd ]; then A="CRT_HIP_LIB=$E/v7wd/libcrt_hip.so CRT_HOST_LIB=$E/v7wd/libcrt_host.so"; else A="X=1"; fi
    env $A timeout -k 10 300 python3 bench.py --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --no-cpu-baseline --no-parity > $OUT/A_${v}_$i.log 2>&1
    echo "round $i $v: still $(grep -o '"kernel_ms_mean": [0-9.]*' $OUT/viewer_still_${v}_$i.json | cut -d' ' -f2) orbit $(grep -o '"kernel_ms_mean": [0-9.]*' $OUT/viewer_orbit_${v}_$i.json | cut -d' ' -f2) A $(grep -o '"ms_per_step": [0-9.]*' $OUT/A_${v}_$i.log | cut -d' ' -f2)"
  done
done
S="T44: T40:T=40 T48:T=48 T52:T=52 T48wd40:T=48,wd=40"
timeout -k 10 300 python3 tools/schedule_sweep.py --world 1 --reps 3 --set $S > $OUT/sweep_C.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 3 --set $S > $OUT/sweep_w8.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 1 --width 1280 --height 720 --spp 256 --reps 3 --set $S > $OUT/sweep_B.jsonl
python3 -c "
import json
for f in ['sweep_C','sweep_w8','sweep_B']:
    print(f, ' '.join('%s %.2f' % (d['name'], d['main_median_ms']) for d in map(json.loads, open('$OUT/%s.jsonl' % f))))"
echo job done
