#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05ac: spatial splits (SBVH, crt_scene_options.spatial_splits) on config B, whose frame is the glass bunny's slowest
# tile (rays inside the mesh), never measured there (C -0.07 %, E +4.7 % at 128 bins).  Prediction: B -3 .. +3 %.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05ac; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u tools/cold_ab.py --configs B --occupancy 0 --trees sah,sbvh --reps 3 > $OUT/B.log 2>&1
grep -v '"rep": 0' $OUT/B.log | cut -c1-200
echo job done
