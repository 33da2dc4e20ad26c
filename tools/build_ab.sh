#!/bin/bash
# Build the native library of another git revision into _ab/lib_<name>.so (for same-box A/B runs
# through MX_GOSSIP_LIB), from a temporary worktree -- the tree's own _native/ build is untouched.
#   bash tools/build_ab.sh <rev> <name>
set -eu
REV=$1; NAME=$2
PKG=270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd
WT=$(mktemp -d /tmp/abwt.XXXX)
git worktree add -q --detach $WT $REV
make -s -C $WT/$PKG -j8 > /dev/null
mkdir -p _ab
cp $WT/$PKG/_native/libmatcha_gossip.so _ab/lib_$NAME.so
git worktree remove --force $WT
echo "_ab/lib_$NAME.so"
