#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04m: variant 7's drain threshold (bits, interactive-loop sweep, wave timelines), then the round-4 final measurement
# set at HEAD: GPU suite, smoke, PMC for C/B/E summarised on the box, default bench + rocprofv3 stats, configs B/E/A,
# RCCL one-rank bench, rank shares, section profile, 2 gloo ranks.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04m; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so bench.py > $OUT/sha.txt
WT=$R/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
timeout -k 10 180 python3 tools/frame_hash.py --big --drain 8 > $OUT/hash_drain8.txt 2>&1
timeout -k 10 180 python3 tools/frame_hash.py --big --drain 1 > $OUT/hash_drain1.txt 2>&1
for d in drain8 drain1; do cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_$d.txt) && echo "$d identical" || echo "$d DIFFERS"; done
F=$(CRT_NO_TORCH=1 python3 -c "import sys; sys.path.insert(0, 'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(map(str, assets.scene_files('cornell_bunny'))))")
for i in 1 2; do
  for d in 0 32 16 8 4 1; do
    timeout -k 10 120 raytracer-cuda_amd/bin/crt_viewer -frames 600 -script still -bvh rebuilt -drain $d $F > $OUT/viewer_still_d${d}_$i.json
  done
  echo "round $i: $(for d in 0 32 16 8 4 1; do echo -n "d$d $(grep -o '"kernel_ms_mean": [0-9.]*' $OUT/viewer_still_d${d}_$i.json | cut -d' ' -f2) "; done)"
done
for d in 0 8 1; do
  CRT_HIP_LIB=$WT timeout -k 10 120 python3 tools/wave_timeline.py --variant 7 --spp 1 --temporal --drain $d >> $OUT/timeline_v7.jsonl 2>> $OUT/timeline.err
done
for d in 0 8 1; do
  timeout -k 10 300 python3 bench.py --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --no-cpu-baseline --no-parity --drain-threshold $d > $OUT/A_d$d.log 2>&1
  echo "A drain $d: $(grep -o '"ms_per_step": [0-9.]*' $OUT/A_d$d.log)"
done
echo drain part done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash tools/pmc.sh gpurun_out/$O/pmc
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
for p in pmc pmc_B pmc_E; do python3 tools/pmc_summary.py gpurun_out/$O/$p profiles/$O/$p > $OUT/summary_$p.log 2>&1; done
cp profiles/roofline_counters.json $OUT/roofline_counters.json
timeout -k 10 400 python3 bench.py --steps 5 > $OUT/bench.log 2>&1
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
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29515 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $OUT/bench_2rank_gloo.log 2>&1
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
echo job done
