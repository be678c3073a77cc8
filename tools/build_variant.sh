#!/bin/bash
# Build an A/B variant of libksched: the persistent-pipeline parts recompiled with extra defines, linked
# with the main build's other objects -> k8s-scheduler_amd/libksched_<name>.so (select it with KSCHED_LIB).
#   bash tools/build_variant.sh spu8 "-DKSCHED_SCREEN_PU=8"
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../k8s-scheduler_amd"
make -s -j8 >/dev/null
mkdir -p build_$name
HIPFLAGS="-O3 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fno-strict-aliasing -fPIC -std=c++17 -I../include -Icsrc -Wall -Wno-unused-result -Wno-unused-value --offload-arch=gfx950"
for p in 0 1 2; do
  /opt/rocm/bin/hipcc $HIPFLAGS $defs -DKSCHED_PIPE_PART=$p -c csrc/ksched_pipe.hip -o build_$name/ksched_pipe$p.o &
done
wait
OBJ="build/ksched_kernels.o build/ksched_commit_spc.o build/ksched_explain.o build_$name/ksched_pipe0.o build_$name/ksched_pipe1.o build_$name/ksched_pipe2.o build/ksched_engine.o build/packer.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libksched_$name.so $OBJ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built k8s-scheduler_amd/libksched_$name.so"
