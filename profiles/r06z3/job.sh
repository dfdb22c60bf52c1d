#!/bin/bash
# r06z3: the round-6 final HEAD end to end: GPU suite, smoke, the default bench line (config C) and its rocprofv3 kernel
# stats, the bench lines of config B, config E and the N = 8 rank share, then the PMC passes of every committed workload
# on this library (so the committed counters carry its hashes).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z3; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
bash tools/gpu_job.sh check $O
cd $R
timeout -k 10 400 python3 bench.py --width 1280 --height 720 --spp 256 > $OUT/B.log 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 > $OUT/E.log 2>&1
timeout -k 10 400 python3 bench.py --share 0 8 > $OUT/S8.log 2>&1
bash tools/pmc.sh gpurun_out/$O/pmc
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
for n in 2 4 8; do
  cd $R
  bash tools/pmc.sh gpurun_out/$O/pmc_s$n --share 0 $n
done
echo job done
