set -u
mkdir -p gpurun_out/pinl; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/pinl
for c in "C1 200" "C2 64"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps 3 $L/librtamd.so $L/librtamd_pinl.so $L/librtamd.so $L/librtamd_pinl.so > $O/$1.log 2>&1 || exit $?
grep -v amdgpu $O/$1.log; done
