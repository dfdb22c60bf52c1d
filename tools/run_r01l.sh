# A/B at 64 spp: current lib (o5 / o6), IEEE-division inv at ray start
set -e
OUT=gpurun_out/r01l
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 400 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4,w4:l4:t2:T40:V4:o6,w4:l4:t2:T36:V4,w4:l4:t2:T44:V4" > $OUT/eval_cur.log 2>&1
CRT_HIP_LIB=$R/raytracer-cuda_amd/lib_exp/inv/libcrt_hip.so timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t2:T40:V4" > $OUT/eval_inv.log 2>&1
echo done
