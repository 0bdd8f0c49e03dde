#!/usr/bin/env bash
# Round 6, call 26: the triangle preset's leaf-postponement threshold q (RT_OPT_TUNE bits 24-27, sixteenths of the
# traversing lanes; the product's default 8 was tuned in round 4 on the 4-wave instance and the reference-shaped tree)
# re-measured on the round's final library (3-wave instance, SAH tree): q = 8, 4, 6, 10, 12.
set -u
cd "$(dirname "$0")/../../.."
L=raytracinginoneweekendinrust_amd/_lib/librtamd.so
timeout -k 10 900 bash tools/ab_session.sh r06_leafq "C4:50 C4" $L $L:0x04000000 $L:0x06000000 $L:0x0a000000 $L:0x0c000000
