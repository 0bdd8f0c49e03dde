# Same-box A/B: mix = the committed kernel, bc = packed slab math with op_sel-broadcast operands
# (the ray's origin and 1/d in three register pairs instead of six splatted pairs) in the
# sphere-BVH presets; then the GPU suite and the bench on bc (the product build).
set -u
mkdir -p gpurun_out/bc; export TMPDIR=/tmp
O=gpurun_out/bc
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_mix.so $L/librtamd_bc.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_bc.so $L/librtamd_mix.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_mix.so $L/librtamd_bc.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_mix.so $L/librtamd_bc.so
run tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd_mix.so $L/librtamd_bc.so
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; exit $rc
