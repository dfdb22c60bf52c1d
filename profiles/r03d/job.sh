# r03d: LDS counters of the leaf-round variants (in-tree vs CRT_LEAF_SELF), section profile at HEAD, default bench
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03d; mkdir -p $OUT
B="python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/lds_A -o p -- $B > $OUT/lds_A.log 2>&1
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/leafself/libcrt_hip.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds_B -o p -- $B > $OUT/lds_B.log 2>&1
cd $R
timeout -k 10 200 python3 tools/section_profile.py --spp 256 > $OUT/section_C256.txt 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-400
python3 - <<'PY'
import csv, glob, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
for v in ("A", "B"):
    tot = {}
    for f in glob.glob(f"{R}/gpurun_out/r03d/lds_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crt_render_kernel<false, 8" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print(v, {k: f"{x:.4g}" for k, x in sorted(tot.items())})
PY
