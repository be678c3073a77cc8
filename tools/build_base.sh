#!/bin/bash
# A/B baseline: the whole library of a committed revision, built in a scratch worktree and copied in-tree as
# k8s-scheduler_amd/libksched_<name>.so (it travels to the GPU box; select it with KSCHED_LIB, which also admits
# the previous ABI version -- ksched/_lib.py).   bash tools/build_base.sh <rev> <name>
set -e
rev=$1; name=$2
cd "$(dirname "$0")/.."
wt=/tmp/ksched_wt_$name
rm -rf $wt && git worktree prune && git worktree add -f --detach $wt $rev >/dev/null
make -s -j8 -C $wt/k8s-scheduler_amd >/dev/null
cp $wt/k8s-scheduler_amd/libksched.so k8s-scheduler_amd/libksched_$name.so
git worktree remove --force $wt
echo "built k8s-scheduler_amd/libksched_$name.so from $(git rev-parse --short $rev)"
