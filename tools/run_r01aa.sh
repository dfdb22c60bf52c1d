# GPU binned-SAH build of the rebuilt tree: tests (incl. 1M triangles), then the whole GPU BVH-build file
OUT=gpurun_out/r01aa
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bvh_build.py -v -s --timeout 300 --timeout-method thread > $OUT/pytest_bvh_build.log 2>&1
set -e
timeout -k 10 600 python3 bench.py --scene cornell_1m --spp 512 --steps 1 --no-cpu-baseline --no-parity > $OUT/bench_E.log 2>&1
echo done
