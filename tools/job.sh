#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05j: where end_to_end_s's scene set-up goes (tools/setup_breakdown.py), configs C and E, with and without torch
# initialised first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05j; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
timeout -k 10 200 python3 tools/setup_breakdown.py > $OUT/C.jsonl 2>&1
timeout -k 10 200 python3 tools/setup_breakdown.py --torch-first > $OUT/C_torch.jsonl 2>&1
timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
cat $OUT/*.jsonl | grep -v amdgpu
echo job done
