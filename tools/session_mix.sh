# Same-box A/B of nf (hoisted offsets), asm (per-trip offsets everywhere) and mix (per-trip in the
# sphere-BVH presets, hoisted in the triangle preset = the product build), then the GPU suite and
# the bench on the product build.
set -u
mkdir -p gpurun_out/mix; export TMPDIR=/tmp
O=gpurun_out/mix
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_nf.so $L/librtamd_asm.so $L/librtamd_mix.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_nf.so $L/librtamd_asm.so $L/librtamd_mix.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_mix.so $L/librtamd_asm.so $L/librtamd_nf.so
run tools/ab_time.py --config C5 --spp 200 --reps 3 $L/librtamd_nf.so $L/librtamd_mix.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-200; exit $rc
