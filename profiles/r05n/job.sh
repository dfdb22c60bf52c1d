#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05n: rank shares with the frame sharded over pixel groups x spp groups (tools/rank_share.py --pixel-groups P): at
# N = 8, P = 2 gives each rank half the tiles at 500 spp instead of every tile at 250.  Predicted: the N = 8 share
# 94.4 % -> ~96 % (the per-wave drain of 500-spp waves) unless 4 tiles per wave slot lengthen the launch's tail.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05n; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
for P in 1 2 4; do
  timeout -k 10 400 python3 tools/rank_share.py --worlds 1 4 8 --reps 2 --pixel-groups $P --all-ranks 8 > $OUT/share_P$P.txt 2>&1
  grep '"world"' $OUT/share_P$P.txt | grep -v efficiency | head -3 | cut -c1-150
  python3 -c "
import json,sys
t=open('$OUT/share_P$P.txt').read(); d=json.loads(t[t.index('{\n'):])
print('P=$P', [(x['world'], x.get('efficiency_vs_n1')) for x in d['rank0']], 'max/min', d.get('all_ranks_max_over_min'), 'slowest rank ms', max(x['end_to_end_ms'] for x in d['all_ranks']))"
done
echo job done
