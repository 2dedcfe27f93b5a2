#!/bin/bash
# Build kernel variants (compile-time knobs of csrc/kernels_rte.hip and csrc/kernels_nn.hip) and time them on the GPU box
# in one process, checking each variant's fluxes bit for bit against the first one.
# Usage: bash tools/solver_variants.sh "name1:-DFOO=1 -DBAR=2" "name2:..." ...
set -e
cd "$(dirname "$0")/.."
PKG=rte-rrtmgp-nn_amd
B=${VAR_DIR:-${TMPDIR:-/tmp}/rrtmgpnn_var}
rm -rf $B; mkdir -p $B
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off"
# sources without tuning knobs are built once
COMMON="api.cpp datafile.cpp kernels_clouds.hip kernels_lw_scat.hip kernels_fluxes.hip"
for f in $COMMON; do /opt/rocm/bin/hipcc $FLAGS -x hip -c $PKG/csrc/$f -o $B/common_${f%.*}.o & done
names=()
for spec in "$@"; do
  n=${spec%%:*}; d=${spec#*:}; names+=($n)
  /opt/rocm/bin/hipcc $FLAGS -fno-slp-vectorize $d -x hip -c $PKG/csrc/kernels_rte.hip -o $B/rte_$n.o &  # as the Makefile
  /opt/rocm/bin/hipcc $FLAGS $d -x hip -c $PKG/csrc/kernels_nn.hip -o $B/nn_$n.o &
  /opt/rocm/bin/hipcc $FLAGS $d -x hip -c $PKG/csrc/kernels_sw_x2.hip -o $B/swx2_$n.o &
done
wait
for n in "${names[@]}"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $B/lib_$n.so $B/common_*.o $B/nn_$n.o $B/rte_$n.o $B/swx2_$n.o -ldl
done
[ -n "${BUILD_ONLY:-}" ] || python3 tools/solver_variants.py $B ${CONFIG:-c3} "${names[@]}"
