#!/bin/bash
# A library variant for same-box A/Bs: hkv_batch.hip and hkv_workload.hip rebuilt with extra defines, linked
# with the in-tree build's other objects into build_ab/NAME/libhermeskv.so.   tools/build_variant.sh NAME "-DX=1 -DY=2"
name=$1; defs=$2; d=build_ab/$name; mkdir -p $d
cd hermes_amd/csrc || exit 1
make -s build/hkv_kernels.o build/hkv_runtime.o build/hkv_hades.o || exit 1
flags="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $flags $defs -c -o ../../$d/hkv_batch.o hkv_batch.hip || exit 1
/opt/rocm/bin/hipcc $flags $defs -c -o ../../$d/hkv_workload.o hkv_workload.hip || exit 1
/opt/rocm/bin/hipcc $flags -shared -o ../../$d/libhermeskv.so ../../$d/hkv_batch.o build/hkv_kernels.o \
  build/hkv_runtime.o ../../$d/hkv_workload.o build/hkv_hades.o || exit 1
rm -f ../../$d/hkv_batch.o ../../$d/hkv_workload.o
