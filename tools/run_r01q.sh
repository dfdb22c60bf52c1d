# occupancy timeline of the headline launch (profiling build, built on the box: lib_exp is not shipped)
set -e
OUT=gpurun_out/r01q
mkdir -p $OUT
bash tools/build_profile_lib.sh wavetimes -DCRT_PROFILE_WAVE_TIMES > $OUT/build.log 2>&1
export CRT_HIP_LIB=$GRAFT_REPO_ROOT/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
timeout -k 10 200 python3 tools/wave_timeline.py > $OUT/timeline_rebuilt_2000.json 2> $OUT/timeline.err
timeout -k 10 200 python3 tools/wave_timeline.py --spp 250 > $OUT/timeline_rebuilt_250.json 2>> $OUT/timeline.err
echo done
