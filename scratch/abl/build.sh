#!/bin/bash
# Ablation library for A/B runs (scratch/ab.sh): a kernels source (default: the committed HEAD
# version of gprx_kernels.hip; or $2) with extra hipcc flags $1, linked with the in-tree objects
# of the other translation units.  Output: libgprx_abl.so (GPRX_LIB selects it).
set -e
cd "$(dirname "$0")"
if [ -n "$2" ]; then cp "$2" gprx_kernels_abl.hip; else git show HEAD:gpr.jl_amd/csrc/gprx_kernels.hip > gprx_kernels_abl.hip; fi
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w -I../../gpr.jl_amd/csrc"
$H $1 -c gprx_kernels_abl.hip -o k.o
L=../../gpr.jl_amd/lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libgprx_abl.so k.o $L/gprx_lbfgs.o $L/gprx_projection.o $L/gprx_api.o
