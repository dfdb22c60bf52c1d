#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04e: (1) the unit-sphere rejection cap against HEAD~'s build (base) and cap 0; (2) L2 hit rate of the XCD-region
# order (r04d measured it slower); (3) VALU counts of the in-tree kernel vs leaf-carry mode 2; (4) a first PC-sampling
# trial (rocprofv3 host_trap) on a short frame, as the last GPU step.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04e; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so raytracer-cuda_amd/lib_exp/*/libcrt_hip.so > $OUT/sha.txt
BASE=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so
C2=$R/raytracer-cuda_amd/lib_exp/carry2/libcrt_hip.so
B="python3 bench.py --no-cpu-baseline --no-count --no-parity"
for i in 1 2 3; do
  CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$BASE timeout -k 10 300 $B > $OUT/base_$i.log 2>&1
  for c in 0 2 3 4 6; do timeout -k 10 300 $B --rejection-cap $c > $OUT/cap${c}_$i.log 2>&1; done
  for f in base cap0 cap2 cap3 cap4 cap6; do echo "$f round $i: $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/${f}_$i.log | tail -1)"; done
done
P1="python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity"
CTR="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
CTR2="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/l2_E_$x -o p -- \
      $P1 --scene cornell_1m --spp 512 --xcd-regions $x > $OUT/l2_E_$x.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/l2_C_$x -o p -- \
      $P1 --xcd-regions $x > $OUT/l2_C_$x.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/sq1_intree -o p -- $P1 > $OUT/sq1_intree.log 2>&1
CRT_HIP_LIB=$C2 timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/sq1_carry2 -o p -- $P1 --carry 16 63 > $OUT/sq1_carry2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $CTR2 --output-format csv -d $OUT/sq2_intree -o p -- $P1 > $OUT/sq2_intree.log 2>&1
CRT_HIP_LIB=$C2 timeout -s KILL 120 rocprofv3 --pmc $CTR2 --output-format csv -d $OUT/sq2_carry2 -o p -- $P1 --carry 16 63 > $OUT/sq2_carry2.log 2>&1
cd $R
python3 - <<'PY'
import csv, glob, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for d in ("l2_C_0", "l2_C_1", "l2_E_0", "l2_E_1", "sq1_intree", "sq1_carry2", "sq2_intree", "sq2_carry2"):
    tot = {}
    for f in glob.glob(f"{R}/gpurun_out/r04e/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crt_render_kernel<false, 8" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 0)
    extra = f" L2 hit {h / (h + m):.4f}" if h + m else ""
    print(d + extra, {k: f"{v:.5g}" for k, v in sorted(tot.items())})
PY
timeout -k 10 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || true
grep -i -B1 -A4 "pc_sampl\|pc sampl" $OUT/list_avail.txt | head -30 || true
cd /tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 --output-format csv -d $OUT/pcs -o pcs -- \
    python3 $R/bench.py --width 1280 --height 720 --spp 64 --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity \
    > $OUT/pcs.log 2>&1
ls -la $OUT/pcs | head
echo job done
