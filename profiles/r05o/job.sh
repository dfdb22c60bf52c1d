#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05o: the host loader's set-up work: the OBJ parse in up to 16 runs of whole lines, the loader's per-face, per-vertex
# and bounds loops on host threads, no copy of the mesh data.  Predicted: config E's load (0.18 s) -> ~0.08 s;
# scene arrays and frames unchanged.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05o; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_A.txt 2>&1
B="CRT_SKIP_ABI_CHECK=1 CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_hip.so CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_exp/base/libcrt_host.so"
env $B timeout -k 10 300 python3 tools/frame_hash.py --big > $OUT/hash_base.txt 2>&1
cmp <(grep -v amdgpu $OUT/hash_A.txt) <(grep -v amdgpu $OUT/hash_base.txt) && echo "hashes identical" | tee $OUT/hash_cmp.txt
CRT_SETUP_TRACE=1 timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline --no-parity > $OUT/E.log 2>&1
timeout -k 10 400 python3 bench.py --steps 3 --no-cpu-baseline --no-parity > $OUT/C.log 2>&1
grep -v amdgpu $OUT/E_torch.jsonl | head -36
for f in E C; do tail -1 $OUT/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["end_to_end"]["end_to_end_s"], d["setup"])' $f; done
echo job done
