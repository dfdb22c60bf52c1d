set -e
O=gpurun_out/ts2
mkdir -p $O
timeout -k 10 900 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l3:t2:T40,w4:l2:t1:T40,w4:l2:t2:T40,w4:l3:t1:T40,w4:l3:t1.5:T40,w4:l4:t1:T40,w4:l4:t2:T40,w4:l2:t1:T48,w4:l3:t2:T48,w4:l3:t2:T32" > $O/eval.log 2>&1
echo done
