#!/bin/bash
# Build an A/B profiling variant of libcrt_hip.so into raytracer-cuda_amd/lib_exp/<name>/ with extra -D flags.
# Usage: tools/build_profile_lib.sh <name> -DFLAG ...   then run with CRT_HIP_LIB=<that path>/libcrt_hip.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
out=$R/raytracer-cuda_amd/lib_exp/$name
mkdir -p $out
cd $R/raytracer-cuda_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-result -munsafe-fp-atomics -fno-slp-vectorize "$@" \
  -I../include -Icsrc -Ihost -shared -o $out/libcrt_hip.so -x hip csrc/crt_hip.hip csrc/crt_bvh_build.hip \
  -Wl,-soname,libcrt_hip.so -Wl,--version-script=csrc/exports.map
echo $out/libcrt_hip.so
