#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04j: the temporal tile order for variant 7 (the interactive loop's 1-spp frames): bits, wave timelines with and
# without it, the interactive loop with and without it; variant 8 against HEAD's build (base) as a check.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04j; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/*/libcrt_hip.so > $OUT/sha.txt
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so; export CRT_HOST_LIB_BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so
WT=$R/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_viewer.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_viewer.log 2>&1
tail -1 $OUT/pytest_viewer.log
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$BASE CRT_HOST_LIB=$CRT_HOST_LIB_BASE timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_base.txt) && echo "hashes identical" || echo "HASHES DIFFER"
for t in "" "--temporal" "" "--temporal"; do
  CRT_HIP_LIB=$WT timeout -k 10 120 python3 tools/wave_timeline.py --variant 7 --spp 1 $t >> $OUT/timeline.jsonl 2>> $OUT/timeline.err
done
python3 -c "
import json
for l in open('$OUT/timeline.jsonl'):
    d=json.loads(l); print(d['temporal'], d['kernel_ms'], d['span_ms'], d['occupancy_efficiency'], d['tail_ms'])"
F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
for i in 1 2; do
  for s in still orbit; do
    timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script $s -bvh rebuilt $F > $OUT/viewer_${s}_temporal_$i.json
    timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script $s -bvh rebuilt -no-temporal $F > $OUT/viewer_${s}_row_$i.json
    echo "$s round $i: temporal $(grep -o '"fps": [0-9.]*' $OUT/viewer_${s}_temporal_$i.json), row $(grep -o '"fps": [0-9.]*' $OUT/viewer_${s}_row_$i.json)"
  done
done
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2; do
  CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$BASE CRT_HOST_LIB=$CRT_HOST_LIB_BASE timeout -k 10 300 $B > $OUT/C_base_$i.log 2>&1
  timeout -k 10 300 $B > $OUT/C_new_$i.log 2>&1
  for f in C_base C_new; do echo "$f round $i: $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
S="base: crit0:crit=0 crit512:crit=512 crit2k:crit=2048 crit4k:crit=4096 lanes8:lanes=8 lanes24:lanes=24 T40:T=40 T48:T=48 occ6:occ=6 stride1:stride=1"
for w in 8 4; do
  timeout -k 10 300 python3 tools/schedule_sweep.py --world $w --reps 3 --set $S > $OUT/sweep_w$w.jsonl
done
cat $OUT/sweep_w8.jsonl | cut -c1-200
for spp in 250 2000; do
  CRT_HIP_LIB=$WT timeout -k 10 150 python3 tools/wave_timeline.py --variant 8 --spp $spp >> $OUT/timeline_v8.jsonl 2>> $OUT/timeline.err
done
echo job done
