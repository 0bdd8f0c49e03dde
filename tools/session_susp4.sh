# RT_SUSPEND 20 / 24 / 28 for C4's 3-wave instance (follow-up of session_susp3.sh).
set -u
mkdir -p gpurun_out/susp3; export TMPDIR=/tmp
O=gpurun_out/susp3
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_s24.so $L/librtamd_s20.so $L/librtamd_s28.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_s28.so $L/librtamd_s20.so $L/librtamd_s24.so
} > $O/ab2.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab2.log; exit $rc
