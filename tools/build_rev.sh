#!/bin/bash
# A/B of the persistent pipeline against a committed revision: rev's csrc/ksched_pipe.hip (and the headers it
# includes) compiled into k8s-scheduler_amd/libksched_<name>.so, linked with the current build's other objects
# (the host ABI -- PersistArgs, PipeLaunch -- must be the same).  Select it with KSCHED_LIB (tools/ab_run.sh).
#   bash tools/build_rev.sh <rev> <name>
set -e
rev=$1; name=$2
cd "$(dirname "$0")/.."
src=/tmp/ksched_rev_$name
rm -rf $src && mkdir -p $src/csrc
for f in $(git ls-tree --name-only $rev k8s-scheduler_amd/csrc/); do git show $rev:$f > $src/csrc/$(basename $f); done
cd k8s-scheduler_amd
make -s -j8 >/dev/null
mkdir -p build_$name
HIPFLAGS="-O3 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fPIC -std=c++17 -I../include -I$src/csrc -Wall -Wno-unused-result -Wno-unused-value --offload-arch=gfx950"
for p in 0 1 2; do
  /opt/rocm/bin/hipcc $HIPFLAGS -DKSCHED_PIPE_PART=$p -c $src/csrc/ksched_pipe.hip -o build_$name/ksched_pipe$p.o &
done
wait
OBJ="build/ksched_kernels.o build/ksched_commit_spc.o build/ksched_explain.o build_$name/ksched_pipe0.o build_$name/ksched_pipe1.o build_$name/ksched_pipe2.o build/ksched_engine.o build/packer.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libksched_$name.so $OBJ -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built k8s-scheduler_amd/libksched_$name.so from $rev"
