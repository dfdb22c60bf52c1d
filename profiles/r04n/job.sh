#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04n: experiment, not in the tree: variant 8's waves pass at a fraction of their live lanes once fewer than the
# regeneration threshold still have samples (profiles/r04n/wave_drain.patch, built as lib_exp/wd16, wd32, wd48 with
# -DCRT_WAVE_DRAIN=16/32/48). Bits, then config C, config B and the N = 8 rank share, interleaved with the in-tree build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04n; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
E=$R/raytracer-cuda_amd/lib_exp
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so $E/wd*/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$E/wd32/libcrt_hip.so CRT_HOST_LIB=$E/wd32/libcrt_host.so timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_wd32.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_wd32.txt) && echo "wd32 identical" || echo "wd32 DIFFERS"
run() {   # label lib args...
  local l=$1 lib=$2; shift 2
  if [ "$lib" = "-" ]; then timeout -k 10 300 "$@"; else CRT_HIP_LIB=$E/$lib/libcrt_hip.so CRT_HOST_LIB=$E/$lib/libcrt_host.so timeout -k 10 300 "$@"; fi
}
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2; do
  for lib in - wd16 wd32 wd48; do
    n=${lib/-/intree}
    run C $lib $B --steps 3 > $OUT/C_${n}_$i.log 2>&1
    run B $lib $B --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_${n}_$i.log 2>&1
    run S $lib python3 tools/schedule_sweep.py --world 8 --reps 2 --set base: > $OUT/w8_${n}_$i.jsonl 2>&1
    echo "round $i $n: C $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/C_${n}_$i.log | tail -1 | cut -d' ' -f2) B $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/B_${n}_$i.log | tail -1 | cut -d' ' -f2) w8 $(grep -o '"main_median_ms": [0-9.]*' $OUT/w8_${n}_$i.jsonl | cut -d' ' -f2)"
  done
done
echo job done
