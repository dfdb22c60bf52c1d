# GPU mesh BVH build tests; interactive loop (row 2): GPU tests incl. the viewer, then frame-time
# runs of the headless loop.  A test failure (pytest rc 1) does not stop the script; a crash / timeout does.
OUT=gpurun_out/r01p
mkdir -p $OUT
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bvh_build.py -v -s --timeout 240 --timeout-method thread > $OUT/pytest_bvh_build.log 2>&1
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_viewer.py -v --timeout 240 --timeout-method thread > $OUT/pytest_viewer.log 2>&1
set -e
FILES=$(python3 -c "import sys; sys.path.insert(0,'raytracer-cuda_amd'); from crt_amd import assets; print(' '.join(assets.scene_files('cornell_bunny')))")
V=raytracer-cuda_amd/bin/crt_viewer
timeout -k 10 120 $V -frames 600 -script still -bvh rebuilt $FILES > $OUT/viewer_still_rebuilt.json
timeout -k 10 120 $V -frames 600 -script still -bvh reference $FILES > $OUT/viewer_still_reference.json
timeout -k 10 120 $V -frames 600 -script orbit -bvh rebuilt $FILES > $OUT/viewer_orbit_rebuilt.json
timeout -k 10 120 $V -frames 600 -script walk -bvh rebuilt $FILES > $OUT/viewer_walk_rebuilt.json
timeout -k 10 120 $V -frames 600 -script still -bvh rebuilt -accumulate -o $OUT/accumulated_600spp.png $FILES > $OUT/viewer_accumulate_rebuilt.json
timeout -k 10 120 $V -frames 3 -script hq -bvh rebuilt -o $OUT/hq_2000spp.png $FILES > $OUT/viewer_hq_rebuilt.json
timeout -k 10 120 $V -w 1280 -frames 600 -script still -bvh rebuilt $FILES > $OUT/viewer_still_rebuilt_720p.json
echo done
