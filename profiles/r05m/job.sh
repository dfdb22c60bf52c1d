#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05m: scene set-up work: the GPU SAH build's bounds / bins per workgroup chunk (LDS bins), the host emission, triangle
# and shading records on up to 16 threads.  Predicted: config E's rebuilt-tree creation 0.34 s -> ~0.17 s (SAH kernels
# 100 -> ~35 ms, emission 76 -> ~25 ms, records 48 -> ~10 ms); trees, scene arrays and frames unchanged.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05m; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bvh_build.py tests/test_gpu_rebuilt.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
B="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_A.txt 2>&1
env $B timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp <(grep -v amdgpu $OUT/hash_A.txt) <(grep -v amdgpu $OUT/hash_base.txt) && echo "hashes identical" | tee $OUT/hash_cmp.txt
CRT_SETUP_TRACE=1 timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o setup -- \
    python3 $R/tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_prof.log 2>&1
cd $R
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline --no-parity > $OUT/E.log 2>&1
timeout -k 10 400 python3 bench.py --steps 3 --no-cpu-baseline --no-parity > $OUT/C.log 2>&1
grep -v amdgpu $OUT/E_torch.jsonl | head -40
for f in E C; do tail -1 $OUT/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["end_to_end"], d["setup"])' $f; done
echo job done
