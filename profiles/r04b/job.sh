#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04a: round-4 first check at HEAD: GPU suite (incl. RCCL one-rank and shipped-instantiation-vs-oracle tests), smoke,
# default bench, bench through torchrun + RCCL at one rank, per-rank shares at N = 1/2/4/8, section profile at HEAD,
# PMC passes for configs B and E, B/E benches with parity, rocprofv3 kernel stats; leaf-pair carry bits + A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04a; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --steps 5 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/bench_rccl1.log 2>&1
tail -1 $OUT/bench_rccl1.log | cut -c1-300
timeout -k 10 300 python3 tools/rank_share.py > $OUT/rank_share.txt 2>&1
timeout -k 10 300 python3 tools/section_profile.py --spp 256 > $OUT/section_C256.txt 2>&1
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
timeout -k 10 300 python3 bench.py --width 1280 --height 720 --spp 256 --steps 5 --no-cpu-baseline > $OUT/B.log 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline > $OUT/E.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
cd $R
for f in bench bench_rccl1 B E; do echo "$f: $(tail -1 $OUT/$f.log | cut -c1-200)"; done
# leaf-pair carry (CRT_LEAF_CARRY build, tools/build_profile_lib.sh carry -DCRT_LEAF_CARRY=1): bits, pair fill, A/B
CL=raytracer-cuda_amd/lib_exp/carry/libcrt_hip.so
timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
CRT_HIP_LIB=$R/$CL timeout -k 10 200 python3 tools/frame_hash.py --big > $OUT/hash_carry.txt 2>&1
cmp <(grep -v amdgpu.ids $OUT/hash_intree.txt) <(grep -v amdgpu.ids $OUT/hash_carry.txt) && echo "carry: hashes identical" || echo "carry: HASHES DIFFER"
CRT_HIP_LIB=$R/$CL timeout -k 10 300 python3 tools/section_profile.py --spp 256 > $OUT/section_C256_carry.txt 2>&1
bash tools/gpu_job.sh ab $O/ab $CL 3
for f in $OUT/ab/bench_*.log; do echo "$(basename $f): $(grep -o '"main_kernel_ms": [0-9.]*' $f | tail -1)"; done
echo job done
