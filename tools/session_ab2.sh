# Same-box A/B: cur = this commit, G = cur with the per-sample segment counter restored,
# D = cur with philox_block inlined in kernel.hip's instances too (the triangle preset).
set -u
mkdir -p gpurun_out/ab2; export TMPDIR=/tmp
O=gpurun_out/ab2
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_cur.so $L/librtamd_G.so $L/librtamd_D.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_D.so $L/librtamd_G.so $L/librtamd_cur.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_cur.so $L/librtamd_G.so $L/librtamd_D.so
run tools/ab_time.py --config C5 --spp 200 --reps 3 $L/librtamd_cur.so $L/librtamd_G.so $L/librtamd_D.so
run tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd_cur.so $L/librtamd_G.so $L/librtamd_D.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
