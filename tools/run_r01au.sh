# validation of HEAD after the packed-FMA slab test: full GPU suite, smoke, bench + rocprofv3 kernel stats, PMC traffic, viewer frame times
OUT=gpurun_out/r01au
R=$GRAFT_REPO_ROOT
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1
FILES=$(python3 -c "import sys; sys.path.insert(0,'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(assets.scene_files('cornell_bunny')))")
V=raytracer-cuda_amd/bin/crt_viewer
timeout -k 10 120 $V -frames 600 -script still -bvh rebuilt $FILES > $OUT/viewer_still_rebuilt.json
timeout -k 10 120 $V -frames 600 -script orbit -bvh rebuilt $FILES > $OUT/viewer_orbit_rebuilt.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/$OUT/bench_prof.log 2>&1
cd $R
SKIP_SQ=1 bash tools/pmc.sh $OUT/pmc
echo done
