#!/bin/bash
# Build librrtmgpnn.so with extra -D flags into variants/<name>.so (for A/B runs through
# RRTMGPNN_LIB): bash tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -eu
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/rte-rrtmgp-nn_amd
OUT=$ROOT/variants
mkdir -p $OUT /tmp/rrtmgpnn_var_$NAME
cd $PKG
make -s -j8 BUILD_DIR=/tmp/rrtmgpnn_var_$NAME LIB=$OUT/$NAME.so EXTRA_FLAGS="$DEFS" $OUT/$NAME.so
echo "built $OUT/$NAME.so ($DEFS)"
