#!/bin/bash
# Build librrtmgpnn.so variants for A/B runs (through RRTMGPNN_LIB or tools/kernel_ab.py) into variants/<name>.so:
#   bash tools/build_variant.sh <name> "<extra hipcc flags>" [ablation ...]
# The sources are copied to /tmp first; ablations (tools/ablations.py: parity-breaking edits that attribute kernel
# time) are applied to the copy only, so the shipped sources never carry them.
set -eu
NAME=$1; DEFS=${2:-}; shift; [ $# -gt 0 ] && shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/variants
SRC=/tmp/rrtmgpnn_var_$NAME/src
mkdir -p $OUT
rm -rf $SRC && mkdir -p $SRC/rte-rrtmgp-nn_amd $SRC/include
cp -r $ROOT/rte-rrtmgp-nn_amd/csrc $ROOT/rte-rrtmgp-nn_amd/Makefile $SRC/rte-rrtmgp-nn_amd/
cp $ROOT/include/*.h $SRC/include/
[ $# -gt 0 ] && python3 $ROOT/tools/ablations.py $SRC/rte-rrtmgp-nn_amd/csrc "$@"
cd $SRC/rte-rrtmgp-nn_amd
make -s -j8 BUILD_DIR=/tmp/rrtmgpnn_var_$NAME/build LIB=$OUT/$NAME.so EXTRA_FLAGS="$DEFS" $OUT/$NAME.so
echo "built $OUT/$NAME.so (flags: $DEFS; ablations: $*)"
