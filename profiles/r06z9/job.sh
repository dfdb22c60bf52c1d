#!/bin/bash
# r06z9: the final HEAD's GPU suite and smoke, as the driver will run them at round end.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r06z9; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo job done
