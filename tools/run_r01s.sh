# variant 7 (persistent pixel queue, probe-cost tile order): parity tests, A/B at 64 spp, bench, wave timeline
OUT=gpurun_out/r01s
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k persistent -v --timeout 240 --timeout-method thread > $OUT/pytest_persistent.log 2>&1
grep -q "failed" $OUT/pytest_persistent.log && { echo "persistent tests failed"; exit 1; }
set -e
timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V7:o6,w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V7:o6" > $OUT/eval_v7.log 2>&1
timeout -k 10 400 python3 bench.py --kernel-variant 7 --no-cpu-baseline > $OUT/bench_v7.log 2>&1
bash tools/build_profile_lib.sh wavetimes -DCRT_PROFILE_WAVE_TIMES > $OUT/build.log 2>&1
CRT_HIP_LIB=$GRAFT_REPO_ROOT/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so timeout -k 10 200 python3 tools/wave_timeline.py --variant 7 > $OUT/timeline_v7_2000.json 2> $OUT/timeline.err
echo done
