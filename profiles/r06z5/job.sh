#!/bin/bash
# r06z5: rocprofv3 kernel stats of config B's and config E's bench lines at the final HEAD (library 77a5ac17), next to
# r06z3's config-C summary.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z5; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_B -o B -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --width 1280 --height 720 --spp 256 --steps 5 > $OUT/B_prof.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_E -o E -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --scene cornell_1m --spp 512 --steps 5 > $OUT/E_prof.log 2>&1
echo job done
