#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04k: final measurement set, part 1, at HEAD (crt_hip.hip with the temporal tile order): GPU suite, frame hashes,
# smoke, PMC passes for configs C, B and E summarised on the box (so this job's bench line carries current counters),
# the default bench (CPU baseline + parity) and the rocprofv3 kernel stats of the bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04k; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash tools/pmc.sh gpurun_out/$O/pmc
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
for p in pmc pmc_B pmc_E; do python3 tools/pmc_summary.py gpurun_out/$O/$p profiles/$O/$p > $OUT/summary_$p.log 2>&1; done
cp profiles/roofline_counters.json $OUT/roofline_counters.json
timeout -k 10 400 python3 bench.py --steps 5 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
echo job done
