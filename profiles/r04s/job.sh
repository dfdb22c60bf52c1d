#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04s: (1) the wave drain for the threaded-BVH variants 2/3/10 (profiles/r04s/v10_wave_drain.patch, built as
# lib_exp/v10wd, not in the tree): bits and the reference-BVH frame (variant 10, the bench's parity path) interleaved
# with the in-tree build; (2) config B's critical tiles re-swept with the wave drain on.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04s; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
E=$R/raytracer-cuda_amd/lib_exp
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so $E/v10wd/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$E/v10wd/libcrt_hip.so CRT_HOST_LIB=$E/v10wd/libcrt_host.so timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_v10wd.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_v10wd.txt) && echo "v10wd identical" || echo "v10wd DIFFERS"
BB="python3 bench.py --no-cpu-baseline --no-count --no-parity --bvh reference"
for i in 1 2; do
  for v in intree v10wd; do
    if [ $v = v10wd ]; then L="CRT_HIP_LIB=$E/v10wd/libcrt_hip.so CRT_HOST_LIB=$E/v10wd/libcrt_host.so"; else L="X=1"; fi
    env $L timeout -k 10 300 $BB --steps 2 > $OUT/Cref_${v}_$i.log 2>&1
    env $L timeout -k 10 300 $BB --width 1280 --height 720 --spp 256 --steps 3 > $OUT/Bref_${v}_$i.log 2>&1
    echo "round $i $v: C-ref $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/Cref_${v}_$i.log | tail -1 | cut -d' ' -f2) B-ref $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/Bref_${v}_$i.log | tail -1 | cut -d' ' -f2)"
  done
done
S="c1024l16: c1024l12:lanes=12 c1024l20:lanes=20 c1024l24:lanes=24 c2048l16:crit=2048 c512l16:crit=512 c2048l24:crit=2048,lanes=24"
timeout -k 10 300 python3 tools/schedule_sweep.py --world 1 --width 1280 --height 720 --spp 256 --reps 4 --set $S > $OUT/sweep_B.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 3 --set c1024l16: c1024l24:lanes=24 c2048l16:crit=2048 > $OUT/sweep_w8.jsonl
python3 -c "
import json
for f in ['sweep_B','sweep_w8']:
    print(f, ' '.join('%s %.2f' % (d['name'], d['main_median_ms']) for d in map(json.loads, open('$OUT/%s.jsonl' % f))))"
echo job done
