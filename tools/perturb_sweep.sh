#!/usr/bin/env bash
# Code-generation stability sweep ("never-executed code"): builds kernel.hip's own
# instances with each never-executed perturbation block (RT_EXP_DEAD, RT_EXP_PERTURB=1..10; the
# blocks are gated by bit 30 of RT_OPT_TUNE or by a scene property no generated scene has) and
# links each with the product's other objects into _lib/librtamd_<name>.so. Then, on a GPU box:
#   python3 tools/ab_time.py --config C1 --reps 1 _lib/librtamd.so _lib/librtamd_p*.so ...
# Every line must read "image identical" with the product's segment count.
set -eu
cd "$(dirname "$0")/../raytracinginoneweekendinrust_amd/csrc"
jobs="${JOBS:-6}"
names=(dead p1 p2 p3 p4 p5 p6 p7 p8 p9 p10)
flags=("-DRT_EXP_DEAD" "-DRT_EXP_PERTURB=1" "-DRT_EXP_PERTURB=2" "-DRT_EXP_PERTURB=3" "-DRT_EXP_PERTURB=4"
       "-DRT_EXP_PERTURB=5" "-DRT_EXP_PERTURB=6" "-DRT_EXP_PERTURB=7" "-DRT_EXP_PERTURB=8" "-DRT_EXP_PERTURB=9"
       "-DRT_EXP_PERTURB=10")
for i in "${!names[@]}"; do
    make variant_main NAME="${names[$i]}" VFLAGS="${flags[$i]}" > "/tmp/perturb_${names[$i]}.log" 2>&1 &
    while [ "$(jobs -r | wc -l)" -ge "$jobs" ]; do sleep 1; done
done
wait
ls -1 ../_lib/librtamd_dead.so ../_lib/librtamd_p*.so
