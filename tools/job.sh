#!/bin/bash
# r06m (second call): frame means by sample position (tools/position_means.py): 8 families x 8 consecutive blocks of
# 250 samples (the renders continue the RNG state), seeds 41 and 43.  Is the first block of every stream different
# from the later ones (a position effect), or are whole streams offset (a family effect), or neither (chance)?
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06m; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u tools/position_means.py > $OUT/position_means.jsonl 2> $OUT/pm.err
echo job done
