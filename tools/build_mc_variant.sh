#!/usr/bin/env bash
# The C1/C2/C3 translation unit (kernel_mc.hip) rebuilt with other device-compiler flags and linked with the
# product's other objects, for same-box A/B (tools/ab_time.py):
#   bash tools/build_mc_variant.sh <name> <flags...>  ->  raytracinginoneweekendinrust_amd/_lib/librtamd_<name>.so
# The product's own mc flags are not added: pass the whole scheduling choice (e.g. -mllvm -misched=...).
set -eu
cd "$(dirname "$0")/../raytracinginoneweekendinrust_amd/csrc"
name="$1"
shift
L=../_lib
mkdir -p "$L/obj_$name"
# the device half alone takes the flags (an -mllvm scheduler name exists only in the AMDGPU backend), then
# the host half embeds that fat binary, as the HIP driver does in one step
F="-O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Wextra -Wno-unused-parameter -Wno-unused-function \
    --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc -fno-slp-vectorize"
/opt/rocm/lib/llvm/bin/clang++ -x hip $F --cuda-device-only "$@" -c kernel_mc.hip -o "$L/obj_$name/kernel_mc.hipfb"
/opt/rocm/lib/llvm/bin/clang++ -x hip $F --cuda-host-only -Xclang -fcuda-include-gpubinary \
    -Xclang "$L/obj_$name/kernel_mc.hipfb" -c kernel_mc.hip -o "$L/obj_$name/kernel_mc.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$L/librtamd_$name.so" $L/obj/kernel.o "$L/obj_$name/kernel_mc.o" \
    $L/obj/kernel_flat.o $L/obj/output.o $L/obj/gather.o $L/obj/bvh_build.o $L/obj/lower.o $L/obj/scenes.o $L/obj/capi.o
echo "$L/librtamd_$name.so"
