#!/bin/bash
# PMC passes for the render kernel (run on the GPU box from the repo root). Each pass is its own rocprofv3 run with
# counters only (no sys/runtime trace) and within the per-block slot limits (MI355X_MICROARCH.md §rocprofv3 PMC slots:
# 8 SQ, 4 TCC with FETCH_SIZE taking 3 and WRITE_SIZE 2, 4 TCP, 2 GRBM).  One timed frame per pass; the summary is
# made on the CPU side by tools/pmc_summary.py.
# Usage: tools/pmc.sh OUTDIR [extra bench args]
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
sha256sum $R/raytracer-cuda_amd/csrc/crt_hip.hip > $R/$OUT/kernel_sha.txt
# the library the passes load (CRT_HIP_LIB or the in-tree build): bench.py checks the counters against it
sha256sum ${CRT_HIP_LIB:-$R/raytracer-cuda_amd/lib/libcrt_hip.so} > $R/$OUT/library_sha.txt
python3 $R/bench.py --print-workload-key "$@" > $R/$OUT/workload_key.txt
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity"
run() { name=$1; shift; ctrs="$1"; shift
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $R/$OUT/$name -o p -- $B "$@" > $R/$OUT/$name.log 2>&1; }
run fetch "FETCH_SIZE GRBM_GUI_ACTIVE" "$@"
run write "WRITE_SIZE" "$@"
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" "$@"
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum" "$@"
run tcp "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE" "$@"
echo pmc done
