#!/bin/bash
# The host-side code under AddressSanitizer + UndefinedBehaviorSanitizer, and the host library under ThreadSanitizer
# (SURVEY §5): builds libcrt_host.so and the
# oracle with -fsanitize=address,undefined (`make asan` in both directories), then runs the CPU tests that drive them
# with the sanitizer runtimes preloaded into python.  Host code only: GPU sanitizers are not available on this pool.
#   tools/run_asan.sh [LOG]        (default profiles/asan/run.log)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$R/profiles/asan/run.log}
mkdir -p "$(dirname "$LOG")"
make -C "$R/raytracer-cuda_amd" -j8 lib/libcrt_hip.so asan > /dev/null
make -C "$R/oracle" asan > /dev/null
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_asan/libcrt_host.so
export ORACLE_LIB=$R/oracle/_asan/liboracle.so
# leaks: python itself holds its allocations at exit; odr: libstdc++ symbols seen twice through the preload
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
TESTS="tests/test_loader_fuzz.py tests/test_loader_runs.py tests/test_host_parity.py tests/test_image_io.py tests/test_camera_controller.py
       tests/test_oracle.py tests/test_primitives_kat.py"
cd "$R"
{
  echo "# tools/run_asan.sh at $(git rev-parse --short HEAD) ($(date -u +%FT%TZ))"
  echo "# $CRT_HOST_LIB, $ORACLE_LIB; preload $ASAN_RT $UBSAN_RT"
} > "$LOG"
set +e
LD_PRELOAD="$ASAN_RT $UBSAN_RT" python -u -m pytest $TESTS -v -p no:cacheprovider -m "not gpu" >> "$LOG" 2>&1
rc=$?
echo "# exit status $rc" >> "$LOG"
# phase 2: the HIP library's host half, built by hipcc with clang's sanitizers (its own runtime, so a separate process);
# the plain host library and oracle
CLANG_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
echo "# phase 2: CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_asan/libcrt_hip.so, preload $CLANG_RT" >> "$LOG"
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_asan/libcrt_hip.so CRT_HOST_LIB= ORACLE_LIB= LD_PRELOAD="$CLANG_RT" \
    python -u -m pytest tests/test_rebuilt_bvh.py tests/test_loader_fuzz.py tests/test_abi.py -v -p no:cacheprovider \
    -m "not gpu" >> "$LOG" 2>&1
rc2=$?
echo "# exit status $rc2" >> "$LOG"
# phase 3: the host library under ThreadSanitizer (the OBJ parser's runs and the loader's host loops)
make -C "$R/raytracer-cuda_amd" tsan > /dev/null
TSAN_RT=$(gcc -print-file-name=libtsan.so)
echo "# phase 3: CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_tsan/libcrt_host.so, preload $TSAN_RT" >> "$LOG"
CRT_HOST_LIB=$R/raytracer-cuda_amd/lib_tsan/libcrt_host.so ORACLE_LIB= TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0" \
    LD_PRELOAD="$TSAN_RT" python -u -m pytest tests/test_loader_runs.py tests/test_loader_fuzz.py -v -p no:cacheprovider \
    -m "not gpu" >> "$LOG" 2>&1
rc3=$?
echo "# exit status $rc3" >> "$LOG"
tail -4 "$LOG"
[ $rc -eq 0 ] && [ $rc2 -eq 0 ] && [ $rc3 -eq 0 ]
