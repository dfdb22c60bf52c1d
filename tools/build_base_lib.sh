#!/bin/bash
# Build libcrt_hip.so from a git revision's kernel sources (default HEAD) into raytracer-cuda_amd/lib_exp/<name>/ —
# the "B" side of tools/gpu_job.sh ab when the working tree holds the change under test.
# Usage: tools/build_base_lib.sh [name=base] [rev=HEAD]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=${1:-base}; rev=${2:-HEAD}
src=$(mktemp -d)
mkdir -p $src/csrc $R/raytracer-cuda_amd/lib_exp/$name
for f in crt_hip.hip crt_bvh_build.hip crt_device.h crt_sah.h exports.map; do
  git -C $R show $rev:raytracer-cuda_amd/csrc/$f > $src/csrc/$f
done
git -C $R show $rev:include/crt_hip.h > $src/crt_hip.h
cd $R/raytracer-cuda_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result -munsafe-fp-atomics -fno-slp-vectorize \
  -I$src -I$src/csrc -Ihost -shared -o lib_exp/$name/libcrt_hip.so $src/csrc/crt_hip.hip $src/csrc/crt_bvh_build.hip \
  -Wl,-soname,libcrt_hip.so -Wl,--version-script=$src/csrc/exports.map
rm -rf $src
echo $R/raytracer-cuda_amd/lib_exp/$name/libcrt_hip.so
