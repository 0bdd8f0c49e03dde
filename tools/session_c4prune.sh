# What exact triangle-BVH pruning could gain on C4 now (RT_OPT_TUNE bit 20 = prune every BVH,
# NOT exact, an upper bound), next to the exact default; 50 spp and the full frame.
set -u
mkdir -p gpurun_out/c4prune; export TMPDIR=/tmp
O=gpurun_out/c4prune
L=raytracinginoneweekendinrust_amd/_lib/librtamd.so
{
for t in 0 0x100000 0 0x100000; do
  echo "== tune=$t"; RT_TUNE=$t timeout -k 10 200 python -u tools/ab_time.py --config C4 --spp 50 --reps 3 $L || exit 1
done
for t in 0 0x100000; do
  echo "== tune=$t full"; RT_TUNE=$t timeout -k 10 200 python -u tools/ab_time.py --config C4 --reps 1 $L || exit 1
done
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
