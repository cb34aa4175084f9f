#!/bin/bash
# Ablation library: production sources with scratch/abl/gprx_kernels_abl.hip (flags via $1)
set -e
cd "$(dirname "$0")"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w -I../../gpr.jl_amd/csrc"
$H $1 -c gprx_kernels_abl.hip -o k.o
L=../../gpr.jl_amd/lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libgprx_abl.so k.o $L/gprx_lbfgs.o $L/gprx_projection.o $L/gprx_api.o
