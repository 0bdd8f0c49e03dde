#!/usr/bin/env bash
# Build librtamd.so with extra device compiler flags into raytracinginoneweekendinrust_amd/_lib/old/
# for same-box A/B timing (RT_LIBRARY=...). Usage: bash tools/build_variant.sh <name> <flags...>
set -eu
cd "$(dirname "$0")/../raytracinginoneweekendinrust_amd/csrc"
name="$1"
shift
mkdir -p ../_lib/old
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
    -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc "$@" -c kernel.hip -o "/tmp/kernel_$name.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../_lib/old/librtamd_$name.so" "/tmp/kernel_$name.o" \
    ../_lib/obj/output.o ../_lib/obj/bvh_build.o ../_lib/obj/lower.o ../_lib/obj/scenes.o ../_lib/obj/capi.o
echo "raytracinginoneweekendinrust_amd/_lib/old/librtamd_$name.so"
