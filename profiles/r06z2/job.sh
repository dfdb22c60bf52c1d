#!/bin/bash
# r06z2: HEAD with the probe-based occupancy choice (rho > 1.6: occupancy 4 with the row prefetch; else 6; >= 4 tiles
# per slot: 7): GPU suite, smoke, default bench + rocprofv3 stats, config B's bench line, the automatic choice on the
# plain Cornell box and the bunny at 1280x720, then the PMC passes of every committed workload on this library.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z2; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
bash tools/gpu_job.sh check $O
cd $R
timeout -k 10 400 python3 bench.py --width 1280 --height 720 --spp 256 > $OUT/B.log 2>&1
timeout -k 10 300 python3 -u tools/occ_sweep.py --scene cornell --w 1280 --h 720 --spp 256 --occ 0 --rounds 1 > $OUT/auto.jsonl 2>> $OUT/auto.err
timeout -k 10 300 python3 -u tools/occ_sweep.py --scene cornell_bunny --w 1280 --h 720 --spp 256 --occ 0 --rounds 1 >> $OUT/auto.jsonl 2>> $OUT/auto.err
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
