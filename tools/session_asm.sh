# Same-box A/B: nf = the committed kernel (near/far row offsets hoisted: 3 registers live across
# the BVH loop), asm = the offsets rederived each trip from the sign bits (volatile asm ashr).
set -u
mkdir -p gpurun_out/asm; export TMPDIR=/tmp
O=gpurun_out/asm
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_nf.so $L/librtamd_asm.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_asm.so $L/librtamd_nf.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_nf.so $L/librtamd_asm.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_nf.so $L/librtamd_asm.so
run tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd_nf.so $L/librtamd_asm.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
