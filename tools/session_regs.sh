# Same-box A/B: A = HEAD kernel, B = per-sample segment count derived from depth,
# C = B + 6-register Rng; then the block order (RT_OPT_TUNE bit 21) on the other configs.
set -u
mkdir -p gpurun_out/regs; export TMPDIR=/tmp
O=gpurun_out/regs
L=raytracinginoneweekendinrust_amd/_lib/old
run() { echo "== $*"; timeout -k 10 240 python -u "$@" || exit 1; }
{
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_A.so $L/librtamd_B.so $L/librtamd_C.so
run tools/ab_time.py --config C3 --spp 100 --reps 5 $L/librtamd_C.so $L/librtamd_B.so $L/librtamd_A.so
run tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd_A.so $L/librtamd_B.so $L/librtamd_C.so
run tools/ab_time.py --config C2 --spp 64 --reps 3 $L/librtamd_A.so $L/librtamd_B.so $L/librtamd_C.so
run tools/ab_time.py --config C5 --spp 200 --reps 3 $L/librtamd_A.so $L/librtamd_B.so $L/librtamd_C.so
run tools/ab_time.py --config C1 --reps 5 $L/librtamd_A.so $L/librtamd_B.so $L/librtamd_C.so
for c in C4 C5 C2 C1; do
  for t in 0 0x200000; do
    echo "tune=$t"; RT_TUNE=$t run tools/shard_time.py --config $c --n 8 --reps 3
  done
done
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
