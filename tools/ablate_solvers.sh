#!/bin/bash
# Build ablation variants of the solver kernels into /tmp and time them on the GPU box in one process.
# Usage (on the GPU box): bash tools/ablate_solvers.sh
set -e
cd "$(dirname "$0")/.."
PKG=rte-rrtmgp-nn_amd
B=${TMPDIR:-/tmp}/rrtmgpnn_abl
mkdir -p $B
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off"
for v in base NATIVE_EXP NO_REDUCE NO_BARRIER; do
  D=""; [ $v != base ] && D="-DRRTMGPNN_ABL_$v"
  /opt/rocm/bin/hipcc $FLAGS $D -x hip -c $PKG/csrc/kernels_rte.hip -o $B/rte_$v.o &
done
/opt/rocm/bin/hipcc $FLAGS -x hip -c $PKG/csrc/kernels_nn.hip -o $B/nn.o &
/opt/rocm/bin/hipcc $FLAGS -x hip -c $PKG/csrc/api.cpp -o $B/api.o &
wait
for v in base NATIVE_EXP NO_REDUCE NO_BARRIER; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $B/lib_$v.so $B/api.o $B/nn.o $B/rte_$v.o
done
python3 tools/ablate_solvers.py $B
