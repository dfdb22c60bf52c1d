#!/bin/bash
# The current one-off GPU job (overwritten per job; the copy that ran is kept as profiles/<id>/job.sh).
# r04y: round-4 final measurement set, part 1 at HEAD: GPU suite, frame hashes, smoke, default bench (CPU baseline +
# parity), rocprofv3 kernel stats of the bench, PMC passes for configs C, B and E.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=r04y; OUT=$R/gpurun_out/$O; mkdir -p $OUT
cd $R
sha256sum raytracer-cuda_amd/csrc/crt_hip.hip raytracer-cuda_amd/lib/libcrt_hip.so > $OUT/sha.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python3 tools/frame_hash.py --big > $OUT/hash_intree.txt 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --steps 5 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 > $OUT/bench_prof.log 2>&1
cd $R
bash tools/pmc.sh gpurun_out/$O/pmc
bash tools/pmc.sh gpurun_out/$O/pmc_B --width 1280 --height 720 --spp 256
bash tools/pmc.sh gpurun_out/$O/pmc_E --scene cornell_1m --spp 512
echo final part 1 done
# diagnostic after the final set: VALU counts of leaf-carry mode 2 against the in-tree kernel
C2=$R/raytracer-cuda_amd/lib_exp/carry2/libcrt_hip.so
P1="python3 $R/bench.py --steps 1 --warmup 0 --no-count --no-cpu-baseline --no-parity"
CTR="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
CTR2="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
cd /tmp && export TMPDIR=/tmp
CRT_HIP_LIB=$C2 timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/sq1_carry2 -o p -- $P1 --carry 16 63 > $OUT/sq1_carry2.log 2>&1
CRT_HIP_LIB=$C2 timeout -s KILL 120 rocprofv3 --pmc $CTR2 --output-format csv -d $OUT/sq2_carry2 -o p -- $P1 --carry 16 63 > $OUT/sq2_carry2.log 2>&1
echo diag done
