#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05t: the GPU mesh BVH build (the reference's median-split builder) with per-chunk LDS reductions for
# big nodes and one thread per small node (<= 32 triangles).  Predicted: 1M-triangle device build 40 -> ~20 ms; trees
# identical to the host builder's.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05t; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bvh_build.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
grep "1M-triangle" $OUT/pytest.log || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o setup -- \
    python3 $R/tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_prof.log 2>&1
cd $R
CRT_SETUP_TRACE=1 timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline --no-parity > $OUT/E.log 2>&1
grep "mesh BVH\|mesh BVHs" $OUT/E_torch.jsonl | head -4
tail -1 $OUT/E.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("E", d["value"], d["end_to_end"]["end_to_end_s"], d["setup"])'
echo job done
