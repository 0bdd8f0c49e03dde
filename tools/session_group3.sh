# Batch size (RT_OPT_GROUP, 0 = automatic) and suspension min-visits re-checked for the 3-wave C1/C4 instances.
set -u
mkdir -p gpurun_out/group3; export TMPDIR=/tmp
O=gpurun_out/group3
L=raytracinginoneweekendinrust_amd/_lib/librtamd.so
{
for g in 0 4 8 16 32 0; do echo "== C4 group=$g"; RT_GROUP=$g timeout -k 10 200 python -u tools/ab_time.py --config C4 --spp 50 --reps 3 $L || exit 1; done
for g in 0 2 4 8 16 0; do echo "== C1 group=$g"; RT_GROUP=$g timeout -k 10 200 python -u tools/ab_time.py --config C1 --reps 5 $L || exit 1; done
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
