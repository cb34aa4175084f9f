#!/bin/bash
# Variant library for A/B runs (scratch/ab_multi.sh): scratch/var/libgprx_NAME.so from a kernels
# source (default: the committed HEAD version of gprx_kernels.hip) with extra hipcc flags, linked
# with the in-tree objects of the other translation units.  GPRX_LIB selects it at run time.
# usage: scratch/varbuild.sh NAME [kernels.hip|HEAD|HEAD~n] [hipcc flags...]
set -e
cd "$(dirname "$0")"
name=$1; src=${2:-HEAD}; shift; shift || true
mkdir -p var
if [ -f "$src" ]; then cp "$src" var/k_$name.hip; else git show $src:gpr.jl_amd/csrc/gprx_kernels.hip > var/k_$name.hip; fi
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w -I../gpr.jl_amd/csrc"
$H "$@" -c var/k_$name.hip -o var/k_$name.o
L=../gpr.jl_amd/lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/libgprx_$name.so var/k_$name.o $L/gprx_lbfgs.o $L/gprx_projection.o $L/gprx_api.o $L/build_id.o
echo "scratch/var/libgprx_$name.so"
