#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05af (second call): occupancy 5 against 6 on config B with 8 interleaved frames per side, and on a 1600x900
# 256-spp frame (22,500 tiles, also below the occupancy-7 rule's 4 tiles per slot).  Rule stated before the run: make
# 5 the automatic choice below that rule if B's mean main kernel is lower by more than 0.8 % and the 1600x900 frame is
# not slower.  Prediction: B -1 .. -2 %, 1600x900 -1 .. +1 %.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05af; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u tools/cold_ab.py --configs B,M --occupancy 6,5 --reps 8 > $OUT/B_occ_2.log 2>&1
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r05af/B_occ_2.log") if l.startswith("{") and '"rep"' in l]
for cfg in ("B", "M"):
    for oc in (6, 5):
        v = [r["main_kernel_ms"] for r in rows if r["config"] == cfg and r["occ"] == oc and r["rep"] > 0]
        print(cfg, oc, len(v), round(sum(v) / len(v), 3), min(v), max(v))
PY
grep hashes $OUT/B_occ_2.log
echo job done
