#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05q: the GPU SAH build's small nodes (<= 16 items) decided one thread each (k_sah_small), the reduction area for big
# nodes only.  Predicted: E's SAH lap 99 -> ~60 ms (kernels ~47 -> ~20 ms, no 2.7-GB area); trees unchanged.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05q; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bvh_build.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
grep "1M-triangle" $OUT/pytest.log || true
CRT_SETUP_TRACE=1 timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o setup -- \
    python3 $R/tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_prof.log 2>&1
cd $R
timeout -k 10 400 python3 bench.py --scene cornell_1m --spp 512 --steps 3 --no-cpu-baseline --no-parity > $OUT/E.log 2>&1
grep "SAH build (GPU)\|rebuilt tree (all)" $OUT/E_torch.jsonl | head -4
tail -1 $OUT/E.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("E", d["value"], d["end_to_end"]["end_to_end_s"], d["setup"])'
echo job done
