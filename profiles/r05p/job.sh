#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05p: the round-5 final measurement set at HEAD (render kernels = 863e141's ISA; host set-up work since r05h): GPU suite, smoke, PMC for C/B/E
# summarised on the box, the default bench, configs B/E/A, RCCL one-rank bench, rank shares, section profile, the
# interactive loop, 2 gloo ranks, rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05p; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash tools/pmc.sh gpurun_out/$O/pmc
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
for p in pmc pmc_B pmc_E; do python3 tools/pmc_summary.py gpurun_out/$O/$p profiles/$O/$p > $OUT/summary_$p.log 2>&1; done
cp profiles/roofline_counters.json $OUT/roofline_counters.json
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 python3 bench.py --width 1280 --height 720 --spp 256 --steps 5 --no-cpu-baseline > $OUT/B.log 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline > $OUT/E.log 2>&1
timeout -k 10 300 python3 bench.py --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --cpu-threads 1 > $OUT/A.log 2>&1
for f in B E A; do echo "$f: $(tail -1 $OUT/$f.log | cut -c1-160)"; done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29514 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/bench_rccl1.log 2>&1
tail -1 $OUT/bench_rccl1.log | cut -c1-200
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share.txt 2>&1
timeout -k 10 300 python3 tools/section_profile.py --spp 256 > $OUT/section_C256.txt 2>&1
bash tools/gpu_job.sh viewer $O/viewer
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29515 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $OUT/bench_2rank_gloo.log 2>&1
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
echo job done
