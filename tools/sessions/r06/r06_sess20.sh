#!/usr/bin/env bash
# Round 6, call 20: the 4-wave instances keep the Perlin tables in LDS when that costs them no wave
# (make variant_main NAME=perm4 VFLAGS=-DRT_PERM_LDS4=1: host-side launch choice only) against the product,
# on C3 (100 spp and the full frame).
set -u
cd "$(dirname "$0")/../../.."
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 900 bash tools/ab_session.sh r06_perm4 "C3:100 C3" $L/librtamd.so $L/librtamd_perm4.so
