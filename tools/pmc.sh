#!/bin/bash
# PMC passes for the render kernel (run on the GPU box from the repo root). Each pass is its own
# rocprofv3 run with counters only (no sys/runtime trace), per MI355X_MICROARCH.md §HBM / rocprofv3.
# Usage: tools/pmc.sh OUTDIR [extra bench args for the SQ passes]
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity"
run() { name=$1; shift; ctrs="$1"; shift
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $R/$OUT/$name -o p -- $B "$@" > $R/$OUT/$name.log 2>&1; }
[ -z "$SKIP_TRAFFIC" ] && run fetch "FETCH_SIZE"
[ -z "$SKIP_TRAFFIC" ] && run write "WRITE_SIZE"
if [ -z "$SKIP_SQ" ]; then
  run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" "$@"
  run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum" "$@"
  run lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" "$@"
  run tcp "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES" "$@"
fi
echo pmc done
