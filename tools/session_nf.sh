# Same-box A/B: head = the committed kernel, nf = BVH rows loaded in the ray's near/far order
# (no per-child selects); then the GPU tests of the traversal (parity, audit, KATs) on nf.
set -u
mkdir -p gpurun_out/nf; export TMPDIR=/tmp
O=gpurun_out/nf
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_head.so $L/librtamd_nf.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_nf.so $L/librtamd_head.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_head.so $L/librtamd_nf.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_head.so $L/librtamd_nf.so
run tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd_head.so $L/librtamd_nf.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
