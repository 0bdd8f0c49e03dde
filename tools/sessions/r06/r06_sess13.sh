#!/usr/bin/env bash
# Round 6, call 13 (on a92b654 + the sbuf_store template, product md5 a39bbe43...): the C1/C2/C3 unit under two
# other AMDGPU schedulers (tools/build_mc_variant.sh itilp -mllvm -misched=gcn-iterative-ilp, minreg
# -mllvm -misched=gcn-iterative-minreg), and non-temporal sample-buffer stores in the BVH presets only
# (make variant NAME=ntbvh VFLAGS=-DRT_SBUF_NT=2: C2 / C5 back to plain stores), against the product.
set -u
cd "$(dirname "$0")/../../.."
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 900 bash tools/ab_session.sh r06_sched "C3:100 C2:64 C5:64 C1" $L/librtamd.so $L/librtamd_itilp.so \
    $L/librtamd_minreg.so $L/librtamd_ntbvh.so
