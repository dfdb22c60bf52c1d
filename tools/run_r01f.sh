# config E bench (both BVH modes), PMC HBM traffic of the headline launch, 2-rank rehearsal
set -e
R=$GRAFT_REPO_ROOT
O=gpurun_out/r01f
mkdir -p $O
timeout -k 10 600 python3 bench.py --scene cornell_1m --spp 512 --steps 2 --no-cpu-baseline > $O/bench_E_rebuilt.log 2>&1
timeout -k 10 600 python3 bench.py --scene cornell_1m --spp 512 --steps 2 --no-cpu-baseline --bvh reference > $O/bench_E_reference.log 2>&1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --spp 64 --steps 2 --no-cpu-baseline --dist-backend gloo > $O/bench_2rank_gloo.log 2>&1
SKIP_SQ=1 bash tools/pmc.sh $O/pmc
echo done
