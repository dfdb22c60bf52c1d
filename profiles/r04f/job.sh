#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04f: (1) the rejection cap with the reference's loop kept for cap 0 and a wave-uniform capped loop, against the
# pre-cap build (base); (2) the probe stride (subsampled cost probe) at 2000 spp and at a 250-spp rank share;
# (3) variant 7 against 8 at 250 spp; (4) bit checks; (5) a PC-sampling trial (rocprofv3 host_trap) last.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04f; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/base/libcrt_hip.so > $OUT/sha.txt
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -m gpu -x -q -k 'rejection_cap or probe_stride' --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1
tail -1 $OUT/pytest_new.log
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_default.txt 2>&1
timeout -k 10 200 python3 tools/frame_hash.py --big --rejection-cap 4 > $OUT/hash_cap4.txt 2>&1
timeout -k 10 200 python3 tools/frame_hash.py --big --probe-stride 2 > $OUT/hash_ps2.txt 2>&1
for f in cap4 ps2; do cmp $OUT/hash_default.txt $OUT/hash_$f.txt && echo "$f: hashes identical" || echo "$f: HASHES DIFFER"; done
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$BASE timeout -k 10 300 $B > $OUT/base_$i.log 2>&1
  for c in 0 3 4 5; do timeout -k 10 300 $B --rejection-cap $c > $OUT/cap${c}_$i.log 2>&1; done
  for s in 2 4; do timeout -k 10 300 $B --probe-stride $s > $OUT/ps${s}_$i.log 2>&1; done
  for f in base cap0 cap3 cap4 cap5 ps2 ps4; do echo "$f round $i: $(grep -o '"render_ms": [0-9.]*, "probe_sort_ms": [0-9.]*, "main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
for i in 1 2; do
  for s in 1 2 4; do timeout -k 10 300 $B --spp 250 --steps 5 --probe-stride $s > $OUT/s250_ps${s}_$i.log 2>&1; done
  timeout -k 10 300 $B --spp 250 --steps 5 --kernel-variant 7 > $OUT/s250_v7_$i.log 2>&1
  for f in s250_ps1 s250_ps2 s250_ps4 s250_v7; do echo "$f round $i: $(grep -o '"render_ms": [0-9.]*, "probe_sort_ms": [0-9.]*, "main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 --output-format csv -d $OUT/pcs -o pcs -- \
    python3 $R/bench.py --width 1280 --height 720 --spp 64 --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity \
    > $OUT/pcs.log 2>&1
ls -la $OUT/pcs | head
echo job done
