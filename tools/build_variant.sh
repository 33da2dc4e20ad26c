#!/bin/bash
# Build the CURRENT tree's native library with extra compile flags (e.g. -DMX_FLOOR_EARLY=0) into
# abship/lib_<name>.so for a same-box A/B through MX_GOSSIP_LIB (the tree's own _native/ build is
# untouched; abship/ travels to the GPU box -- delete it after the A/B).
#   bash tools/build_variant.sh <name> "<flags>"
set -eu
NAME=$1; FLAGS=$2
PKG=270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd
TMP=$(mktemp -d /tmp/abvar.XXXX)
mkdir -p $TMP/$PKG
cp -r include $TMP/
cp -r $PKG/csrc $PKG/Makefile $TMP/$PKG/
make -s -C $TMP/$PKG -j8 EXTRA="$FLAGS" > /dev/null
mkdir -p abship
cp $TMP/$PKG/_native/libmatcha_gossip.so abship/lib_$NAME.so
rm -rf $TMP
echo "abship/lib_$NAME.so"
