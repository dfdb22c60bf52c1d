# final-state measurements: 2-rank rehearsal (gloo, both ranks on the one GPU), bench, rocprofv3 stats, PMC passes
OUT=gpurun_out/r01ab
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
set -e
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --spp 256 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_2rank_gloo.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
cd $R
bash tools/pmc.sh $OUT/pmc
echo done
