# The suspending walk's lane threshold (RT_SUSPEND, 16 chosen at 4 waves) re-checked for C4's 3-wave instance.
set -u
mkdir -p gpurun_out/susp3; export TMPDIR=/tmp
O=gpurun_out/susp3
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_s16.so $L/librtamd_s8.so $L/librtamd_s24.so $L/librtamd_s32.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_s32.so $L/librtamd_s24.so $L/librtamd_s8.so $L/librtamd_s16.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
