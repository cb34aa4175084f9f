#!/bin/bash
# Variant library for A/B runs (scratch/ab_multi.sh): scratch/var/libgprx_NAME.so built from a git
# revision of the whole csrc tree (default HEAD), or from a kernels source file with the in-tree
# other translation units, with extra hipcc flags.  GPRX_LIB selects it at run time.
# usage: scratch/varbuild.sh NAME [REV|kernels.hip] [hipcc flags...]
set -e
cd "$(dirname "$0")"
name=$1; src=${2:-HEAD}; shift; shift || true
mkdir -p var
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w"
if [ -f "$src" ]; then
  cp "$src" var/k_$name.hip
  $H -I../gpr.jl_amd/csrc "$@" -c var/k_$name.hip -o var/k_$name.o
  L=../gpr.jl_amd/lib
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/libgprx_$name.so var/k_$name.o $L/gprx_lbfgs.o $L/gprx_projection.o $L/gprx_api.o $L/build_id.o
else
  d=var/src_$name; rm -rf $d; mkdir -p $d
  git -C .. archive "$src" gpr.jl_amd/csrc include | tar -x -C $d
  objs=""
  for f in $d/gpr.jl_amd/csrc/*.hip; do
    o=$d/$(basename $f .hip).o
    $H -I$d/gpr.jl_amd/csrc "$@" -c $f -o $o &
    objs="$objs $o"
  done
  for j in $(jobs -p); do wait $j; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/libgprx_$name.so $objs ../gpr.jl_amd/lib/build_id.o
fi
echo "scratch/var/libgprx_$name.so"
