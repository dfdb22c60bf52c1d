# variant 7 with first-block-exclusive waves and lower regen thresholds vs 4 and 8, at 2000 spp; variant 8 timeline
OUT=gpurun_out/r01v
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rebuilt.py -k "persistent or xcd or first_block" -v --timeout 240 --timeout-method thread > $OUT/pytest_order.log 2>&1
grep -q "failed" $OUT/pytest_order.log && { echo "order tests failed"; exit 1; }
set -e
timeout -k 10 700 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V4:o6,w4:l4:t2:T40:V8:o6:P4,w4:l4:t2:T40:V7:o6:P4,w4:l4:t2:T40:V7:o6:P4:F1,w4:l4:t2:T24:V7:o6:P4,w4:l4:t2:T24:V7:o6:P4:F1,w4:l4:t2:T32:V8:o6:P4" > $OUT/eval_v7f_2000.log 2>&1
bash tools/build_profile_lib.sh wavetimes -DCRT_PROFILE_WAVE_TIMES > $OUT/build.log 2>&1
export CRT_HIP_LIB=$GRAFT_REPO_ROOT/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
timeout -k 10 200 python3 tools/wave_timeline.py --variant 8 --persistent-waves 57600 > $OUT/timeline_v8_2000.json 2> $OUT/timeline.err
echo done
