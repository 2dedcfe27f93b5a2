#!/bin/bash
# Register / spill / occupancy summary of every kernel in one source file (compiler view):
#   bash tools/kres.sh csrc/kernels_sw_ck.hip "-DFOO=1" [name-filter]
set -u
SRC=$1; DEFS=${2:-}; FILT=${3:-.}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/rte-rrtmgp-nn_amd
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $DEFS -x hip -c $SRC -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name:/ {n=$NF} / VGPRs:/ {v=$NF} /AGPRs:/ {a=$NF} /ScratchSize/ {sc=$NF} /Occupancy/ {print "vgpr", v, "agpr", a, "scratch", sc, "occ", $NF, n}' |
  c++filt | grep -E -- "$FILT" | cut -c1-220
