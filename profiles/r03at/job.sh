# r03at: round-3 final measurement set (variant 8 at occupancy 7 for C/E, 6 for B; variants 3 and 10 at 6); GPU suite, hashes, default bench + rocprofv3 stats, PMC, configs A/B/E, the interactive loop, 2 gloo ranks
# the interactive loop
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r03at; OUT=$R/gpurun_out/$O; mkdir -p $OUT
git -C $R rev-parse HEAD > $OUT/head.txt 2>/dev/null || true
sha256sum $R/raytracer-cuda_amd/csrc/crt_hip.hip $R/raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -2 $OUT/pytest_gpu.log
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
grep -v amdgpu.ids $OUT/hash_intree.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --steps 5 > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc
timeout -k 10 300 python3 bench.py --width 1280 --height 720 --spp 256 --steps 5 --no-cpu-baseline --no-parity > $OUT/B.log 2>&1
timeout -k 10 300 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline --no-parity > $OUT/E.log 2>&1
timeout -k 10 300 python3 bench.py --scene cornell --width 256 --height 256 --spp 16 --bounces 4 --steps 20 --cpu-threads 1 > $OUT/A.log 2>&1
bash tools/gpu_job.sh viewer $O/viewer
for f in bench B E A; do echo "$f: $(tail -1 $OUT/$f.log | cut -c1-160)"; done
# multi-rank rehearsal of the bench's sharded path at HEAD (gloo, ranks sharing this GPU; RCCL refuses that)
cd $R
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $OUT/bench_2rank_gloo.log 2>&1
tail -1 $OUT/bench_2rank_gloo.log | cut -c1-200
