# cur = product; mcall = kernel.hip's own instances (C1's and C4's 3-wave ones, the replay pass) also
# built with the memory-clause scheduler.
set -u
mkdir -p gpurun_out/mcall; export TMPDIR=/tmp
O=gpurun_out/mcall
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_cur.so $L/librtamd_mcall.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_mcall.so $L/librtamd_cur.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_cur.so $L/librtamd_mcall.so
run tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd_cur.so $L/librtamd_mcall.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
