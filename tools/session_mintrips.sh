# The suspending walk's minimum visits per call before a traversal may stop (RT_SUSP_MIN_TRIPS, 2)
# re-checked for C4's 3-wave instance.
set -u
mkdir -p gpurun_out/mintrips; export TMPDIR=/tmp
O=gpurun_out/mintrips
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_m2.so $L/librtamd_m1.so $L/librtamd_m4.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_m4.so $L/librtamd_m1.so $L/librtamd_m2.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
