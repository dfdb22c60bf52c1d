#!/bin/bash
# Build libcrt_hip.so from a git revision's kernel sources (default HEAD) into raytracer-cuda_amd/lib_exp/<name>/ —
# the "B" side of an A/B run when the working tree holds the change under test (CRT_HIP_LIB=lib_exp/<name>/libcrt_hip.so
# CRT_HOST_LIB=lib_exp/<name>/libcrt_host.so).
# Usage: tools/build_base_lib.sh [name=base] [rev=HEAD] [patch to crt_hip.hip, or -] [extra hipcc flags...]
# (a patch builds an experiment that is not in the tree, e.g. profiles/r04n/wave_drain.patch -DCRT_WAVE_DRAIN=32)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=${1:-base}; rev=${2:-HEAD}; patchf=${3:--}; shift $(( $# < 3 ? $# : 3 ))
src=$(mktemp -d)
mkdir -p $src/csrc $R/raytracer-cuda_amd/lib_exp/$name
for f in crt_hip.hip crt_bvh_build.hip crt_device.h crt_sah.h exports.map; do
  git -C $R show $rev:raytracer-cuda_amd/csrc/$f > $src/csrc/$f
done
git -C $R show $rev:include/crt_hip.h > $src/crt_hip.h
if [ "$patchf" != "-" ]; then patch -s $src/csrc/crt_hip.hip < $patchf; fi
cd $R/raytracer-cuda_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result -munsafe-fp-atomics -fno-slp-vectorize \
  -I$src -I$src/csrc -Ihost -shared -o lib_exp/$name/libcrt_hip.so $src/csrc/crt_hip.hip $src/csrc/crt_bvh_build.hip \
  -Wl,-soname,libcrt_hip.so -Wl,--version-script=$src/csrc/exports.map "$@"
# the host library of the same revision (CRT_HOST_LIB), linked against this libcrt_hip.so: HEAD's host library may
# call entry points an older libcrt_hip.so lacks
git -C $R archive $rev raytracer-cuda_amd/host include | tar -x -C $src
(cd $src/raytracer-cuda_amd && g++ -O2 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I../include -Ihost -shared \
  -o $R/raytracer-cuda_amd/lib_exp/$name/libcrt_host.so host/crt/ImageIO.cpp host/crt/ObjLoader.cpp host/crt/BVHBuild.cpp \
  host/crt/SceneManager.cpp host/crt_host_capi.cpp -L$R/raytracer-cuda_amd/lib_exp/$name -lcrt_hip -Wl,-rpath,'$ORIGIN')
rm -rf $src
echo $R/raytracer-cuda_amd/lib_exp/$name/libcrt_hip.so
