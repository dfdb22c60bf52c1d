#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06i: PMC passes on the round-6 source for the other committed workloads (config B, config E, the N = 2 / 4 / 8 rank-0
# shares), so every roofline_counters.json entry carries the current kernel-source hash.  The binary is the same as
# round 5's, so the per-ray counters should repeat r05p / r06b to the last digit of the instruction counts.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06i; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
for n in 2 4 8; do
  cd $R
  bash tools/pmc.sh gpurun_out/$O/pmc_s$n --share 0 $n
done
echo job done
