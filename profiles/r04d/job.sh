#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04d: XCD-region tile order (crt_renderer_set_xcd_regions): bit-identity test, A/B on configs C and E, L2 hit rate
# with and without; the unit-sphere rejection cap (crt_renderer_set_rejection_cap): bits and an A/B against HEAD's build.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04d; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -m gpu -x -q -k 'xcd or rejection_cap' --timeout 200 --timeout-method thread > $OUT/pytest_xcd.log 2>&1
tail -1 $OUT/pytest_xcd.log
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_off.txt 2>&1
timeout -k 10 200 python3 tools/frame_hash.py --big --xcd-regions 1 > $OUT/hash_on.txt 2>&1
cmp $OUT/hash_off.txt $OUT/hash_on.txt && echo "xcd: hashes identical" || echo "xcd: HASHES DIFFER"
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  timeout -k 10 300 $B --xcd-regions 0 > $OUT/C_off_$i.log 2>&1
  timeout -k 10 300 $B --xcd-regions 1 > $OUT/C_on_$i.log 2>&1
  timeout -k 10 300 $B --scene cornell_1m --spp 512 --xcd-regions 0 > $OUT/E_off_$i.log 2>&1
  timeout -k 10 300 $B --scene cornell_1m --spp 512 --xcd-regions 1 > $OUT/E_on_$i.log 2>&1
  for f in C_off C_on E_off E_on; do echo "$f round $i: $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
timeout -k 10 200 python3 tools/frame_hash.py --big --rejection-cap 3 > $OUT/hash_cap3.txt 2>&1
cmp $OUT/hash_off.txt $OUT/hash_cap3.txt && echo "cap3: hashes identical" || echo "cap3: HASHES DIFFER"
for i in 1 2 3; do
  CRT_HIP_LIB=$BASE timeout -k 10 300 $B > $OUT/base_$i.log 2>&1
  for c in 0 3 4 6; do timeout -k 10 300 $B --rejection-cap $c > $OUT/cap${c}_$i.log 2>&1; done
  for f in base cap0 cap3 cap4 cap6; do echo "$f round $i: $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/l2_E_$x -o p -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity --scene cornell_1m --spp 512 \
      --xcd-regions $x > $OUT/l2_E_$x.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/l2_C_$x -o p -- \
      python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity --xcd-regions $x > $OUT/l2_C_$x.log 2>&1
done
cd $R
python3 - <<'PY'
import csv, glob, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for d in ("l2_C_0", "l2_C_1", "l2_E_0", "l2_E_1"):
    tot = {}
    for f in glob.glob(f"{R}/gpurun_out/r04d/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crt_render_kernel<false, 8" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
    print(d, "L2 hit rate", round(h / max(1, h + m), 4), {k: f"{v:.4g}" for k, v in tot.items()})
PY
echo job done
