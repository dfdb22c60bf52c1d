#!/bin/bash
# One parameterised GPU job for gpurun (run from the repo root on the GPU box). Every GPU step has its own time
# limit and the steps are chained with set -e, so a failing or hung step ends the job.
#
#   tools/gpu_job.sh check OUT            GPU tests, smoke, default bench, rocprofv3 kernel stats of the bench
#   tools/gpu_job.sh bench OUT [ARGS..]   bench.py ARGS, then the same under rocprofv3 --kernel-trace --stats
#   tools/gpu_job.sh ab OUT LIB_B [N] [ARGS..]
#                                         A/B of the in-tree libcrt_hip.so (A) against LIB_B (a build from
#                                         tools/build_profile_lib.sh), N alternating A B rounds of bench.py ARGS
#   tools/gpu_job.sh pmc OUT [ARGS..]     rocprofv3 --pmc passes (tools/pmc.sh) over one bench frame
#   tools/gpu_job.sh l1 OUT               vector-L1 calibration micro-benchmark (tools/probes/l1_probe.hip) + PMC
#   tools/gpu_job.sh libs OUT N LIB ...     N interleaved rounds of the default bench over the in-tree library (A) and
#                                         each LIB (paths to libcrt_hip.so builds, e.g. from tools/build_profile_lib.sh)
#   tools/gpu_job.sh viewer OUT            the interactive loop (bin/crt_viewer): 600 frames of 1 spp at 2560x1440, still
#                                         and orbiting, rebuilt BVH, one JSON line each
#   tools/gpu_job.sh sweep OUT N "label=ARGS" ...
#                                         N interleaved rounds of bench.py, one run per "label=ARGS" set (the args
#                                         after '=' split on spaces); one log per label and round
set -e
MODE=$1; OUT=gpurun_out/$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
case $MODE in
check)
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $R/$OUT/pytest_gpu.log 2>&1
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $R/$OUT/smoke.log 2>&1
  timeout -k 10 400 python3 bench.py > $R/$OUT/bench.log 2>&1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- \
      python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
  ;;
bench)
  timeout -k 10 600 python3 bench.py "$@" > $R/$OUT/bench.log 2>&1
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- \
      python3 $R/bench.py --no-cpu-baseline --no-parity "$@" > $R/$OUT/bench_prof.log 2>&1
  ;;
ab)
  LIBB=$1; N=${2:-2}; shift 2
  for i in $(seq 1 $N); do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity "$@" > $R/$OUT/bench_A$i.log 2>&1
    CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/$LIBB timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity "$@" \
        > $R/$OUT/bench_B$i.log 2>&1
  done
  ;;
pmc)
  bash tools/pmc.sh $OUT "$@"
  ;;
l1)
  # vector-L1 calibration (tools/probes/l1_probe.hip, built on the CPU side): timings, then one PMC pass
  timeout -k 10 120 tools/probes/l1_probe > $R/$OUT/l1_probe.log 2>&1
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE \
      --output-format csv -d $R/$OUT/pmc -o l1 -- $R/tools/probes/l1_probe > $R/$OUT/l1_pmc.log 2>&1
  ;;
libs)
  N=$1; shift
  for i in $(seq 1 $N); do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity > $R/$OUT/A_$i.log 2>&1
    echo "A round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $R/$OUT/A_$i.log)"
    for lib in "$@"; do
      label=$(basename $(dirname $lib))
      CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity > $R/$OUT/${label}_$i.log 2>&1
      echo "$label round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $R/$OUT/${label}_$i.log)"
    done
  done
  ;;
viewer)
  F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
  for s in still orbit; do
    timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script $s -bvh rebuilt $F > $R/$OUT/viewer_${s}_rebuilt.json
  done
  ;;
sweep)
  N=$1; shift
  for i in $(seq 1 $N); do
    for spec in "$@"; do
      label=${spec%%=*}; args=${spec#*=}
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-count --no-parity $args > $R/$OUT/${label}_$i.log 2>&1
      echo "$label round $i: $(grep -o '"render_kernel_ms_avg": [0-9.]*' $R/$OUT/${label}_$i.log)"
    done
  done
  ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
echo "gpu_job $MODE done"
