set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/wfprof3
timeout -k 10 300 python3 -m pytest tests/test_gpu_rebuilt.py -x -q -k "wavefront" > $R/gpurun_out/wfprof3/pytest.log 2>&1
timeout -k 10 300 python3 tools/bvh_eval.py --no-compare --spp 64 --configs "w4:l4:t3:T40,w4:l4:t3:V5:R16,w4:l4:t3:V5:R32" > $R/gpurun_out/wfprof3/eval.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wfprof3/p -o wf -- python3 $R/tools/wf_probe.py 64 16 > $R/gpurun_out/wfprof3/log 2>&1
echo done
