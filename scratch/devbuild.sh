#!/bin/bash
# Variant library from the whole scratch/dev source tree (kernels, API, header), for A/B runs that
# change more than the kernels file: scratch/var/libgprx_NAME.so.  Populate the tree first
# (mkdir -p scratch/dev && cp gpr.jl_amd/csrc/*.hip gpr.jl_amd/csrc/*.h scratch/dev/), edit it, then
# usage: scratch/devbuild.sh NAME [hipcc flags...]
set -e
cd "$(dirname "$0")"
name=$1; shift
mkdir -p var/o_$name
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w -Idev"
objs=""
for f in dev/gprx_kernels.hip dev/gprx_lbfgs.hip dev/gprx_projection.hip dev/gprx_api.hip; do
  o=var/o_$name/$(basename $f .hip).o
  $H "$@" -c $f -o $o &
  objs="$objs $o"
done
for j in $(jobs -p); do wait $j; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/libgprx_$name.so $objs ../gpr.jl_amd/lib/build_id.o
rm -rf var/o_$name
echo "scratch/var/libgprx_$name.so"
