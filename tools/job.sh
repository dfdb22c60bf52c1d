#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r05k: the host stages of scene creation (CRT_SETUP_TRACE=1) for configs C and E, torch initialised first.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r05k; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
CRT_SETUP_TRACE=1 timeout -k 10 200 python3 tools/setup_breakdown.py --torch-first > $OUT/C_torch.jsonl 2>&1
CRT_SETUP_TRACE=1 timeout -k 10 300 python3 tools/setup_breakdown.py --scene cornell_1m --torch-first > $OUT/E_torch.jsonl 2>&1
grep -v amdgpu $OUT/E_torch.jsonl
echo job done
