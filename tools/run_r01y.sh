# variant 8 (work probe): occupancy timeline, regen-threshold sweep at 2000 spp, config E (1M triangles, 512 spp)
OUT=gpurun_out/r01y
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
set -e
timeout -k 10 700 python3 tools/bvh_eval.py --no-compare --spp 2000 --reps 1 --configs "w4:l4:t2:T40:V8:o6,w4:l4:t2:T48:V8:o6,w4:l4:t2:T56:V8:o6,w4:l4:t2:T32:V8:o6,w4:l4:t2:T40:V8:o6" > $OUT/eval_v8_T_2000.log 2>&1
timeout -k 10 600 python3 bench.py --scene cornell_1m --spp 512 --steps 2 --no-cpu-baseline > $OUT/bench_E_v8.log 2>&1
timeout -k 10 600 python3 bench.py --scene cornell_1m --spp 512 --steps 2 --no-cpu-baseline --no-parity --kernel-variant 4 > $OUT/bench_E_v4.log 2>&1
bash tools/build_profile_lib.sh wavetimes -DCRT_PROFILE_WAVE_TIMES > $OUT/build.log 2>&1
export CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
timeout -k 10 200 python3 tools/wave_timeline.py --variant 8 --persistent-waves 57600 > $OUT/timeline_v8w_2000.json 2> $OUT/timeline.err
echo done
