#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r06q: the round-6 HEAD after the profiling switches of r06n-r06p (shipped library byte-identical to r06z's,
# b74f5380): GPU suite, smoke, the default bench line (now with counters_kernel_library_current) and its rocprofv3
# kernel stats, then the PMC passes for every committed workload on this source, so the counters carry its hash.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06q; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
bash tools/gpu_job.sh check $O
cd $R
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
