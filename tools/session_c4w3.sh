# C4 now runs the 3-wave triangle instance: re-check its two per-preset choices made at 4 waves.
# cur = product; v1 = per-trip near-row offsets in the triangle preset too; v2 = Philox inlined there.
set -u
mkdir -p gpurun_out/c4w3; export TMPDIR=/tmp
O=gpurun_out/c4w3
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_cur.so $L/librtamd_v1.so $L/librtamd_v2.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_v2.so $L/librtamd_v1.so $L/librtamd_cur.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_cur.so $L/librtamd_v1.so $L/librtamd_v2.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
