#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04o: the wave drain in the tree (crt_renderer_set_wave_drain, default 48/64): bits, an interleaved A/B against
# 64/64 and against the previous HEAD's build (base = r04m's source), a sweep on B and the N = 8 share; then the
# round-4 final measurement set at HEAD: GPU suite, smoke, PMC for C/B/E summarised on the box, default bench,
# configs B/E/A, RCCL one-rank bench, rank shares, section profile, 2 gloo ranks, rocprofv3 stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04o; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
E=$R/raytracer-cuda_amd/lib_exp
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so $E/base/libcrt_hip.so bench.py > $OUT/sha.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k wave_drain -x -q --timeout 200 --timeout-method thread > $OUT/pytest_wave_drain.log 2>&1
tail -1 $OUT/pytest_wave_drain.log
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
timeout -k 10 180 python3 tools/frame_hash.py --big --wave-drain 64 > $OUT/hash_wd64.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_wd64.txt) && echo "wd64 identical" || echo "wd64 DIFFERS"
BB="python3 bench.py --no-cpu-baseline --no-count --no-parity"
BASE="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$E/base/libcrt_hip.so CRT_HOST_LIB=$E/base/libcrt_host.so"
for i in 1 2; do
  for v in new wd64 base; do
    case $v in new) X=""; P="";; wd64) X="--wave-drain 64"; P="";; base) X=""; P="$BASE";; esac
    env $P timeout -k 10 300 $BB --steps 3 $X > $OUT/C_${v}_$i.log 2>&1
    env $P timeout -k 10 300 $BB --width 1280 --height 720 --spp 256 --steps 5 $X > $OUT/B_${v}_$i.log 2>&1
    echo "round $i $v: C $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/C_${v}_$i.log | tail -1 | cut -d' ' -f2) B $(grep -o '"main_kernel_ms": [0-9.]*' $OUT/B_${v}_$i.log | tail -1 | cut -d' ' -f2)"
  done
done
S="wd48: wd64:wd=64 wd56:wd=56 wd40:wd=40 wd32:wd=32"
timeout -k 10 300 python3 tools/schedule_sweep.py --world 8 --reps 3 --set $S > $OUT/sweep_w8.jsonl
timeout -k 10 300 python3 tools/schedule_sweep.py --world 1 --width 1280 --height 720 --spp 256 --reps 3 --set $S > $OUT/sweep_B.jsonl
cut -c1-120 $OUT/sweep_w8.jsonl $OUT/sweep_B.jsonl
echo ab part done
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
bash tools/gpu_job.sh viewer $O/viewer
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29515 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $OUT/bench_2rank_gloo.log 2>&1
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
echo job done
