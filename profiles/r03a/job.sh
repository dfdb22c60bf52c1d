set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03a; mkdir -p $OUT
L=$R/raytracer-cuda_amd/lib_exp/wavetimes/libcrt_hip.so
CRT_HIP_LIB=$L timeout -k 10 200 python3 tools/wave_timeline.py --w 1280 --h 720 --spp 256 --variant 8 > $OUT/timeline_B.json 2> $OUT/timeline_B.err
CRT_HIP_LIB=$L timeout -k 10 200 python3 tools/wave_timeline.py --w 1280 --h 720 --spp 256 --variant 8 > $OUT/timeline_B2.json 2>> $OUT/timeline_B.err
CRT_HIP_LIB=$L timeout -k 10 300 python3 tools/wave_timeline.py --spp 2000 --variant 8 > $OUT/timeline_C.json 2> $OUT/timeline_C.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --width 1280 --height 720 --spp 256 --steps 5 > $OUT/bench_B.log 2>&1
echo done
