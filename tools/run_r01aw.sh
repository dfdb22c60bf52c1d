# A/B: Möller–Trumbore with paired v_pk_mul/v_pk_add_f32 (lib/, default) vs the scalar form (-DCRT_TRI_SCALAR);
# GPU parity suite on the packed build first, then the headline bench alternated A B A B.
OUT=gpurun_out/r01aw
mkdir -p $OUT
set -e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
S=raytracer-cuda_amd/lib_exp/scalar/libcrt_hip.so
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count > $OUT/bench_pk1.log 2>&1
CRT_HIP_LIB=$PWD/$S timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count > $OUT/bench_sc1.log 2>&1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count --no-parity > $OUT/bench_pk2.log 2>&1
CRT_HIP_LIB=$PWD/$S timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-count --no-parity > $OUT/bench_sc2.log 2>&1
echo done
