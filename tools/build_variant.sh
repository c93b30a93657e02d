#!/bin/bash
# Experiment builds: vectorscan_amd/libvsa_<name>.so with extra -D flags on
# the kernels (load with VSA_LIB_VARIANT=libvsa_<name>.so).
#   tools/build_variant.sh exp4 -DEXP_U=4
#   KSRC=/path/to/kernels.hip tools/build_variant.sh prev   (another kernels source)
set -e
name=$1; shift
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-parameter -Iinclude"
C=vectorscan_amd/csrc
mkdir -p /tmp/vsa_variant_$name
$H "$@" -I$C -c ${KSRC:-$C/kernels.hip} -o /tmp/vsa_variant_$name/kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $C/compile.o $C/flood.o $C/hs_lit.o \
    /tmp/vsa_variant_$name/kernels.o $C/runtime.o $C/plan.o $C/dropin.o $C/batcher.o \
    -o vectorscan_amd/libvsa_$name.so
echo built vectorscan_amd/libvsa_$name.so
