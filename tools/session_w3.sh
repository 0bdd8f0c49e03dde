# The 3-wave instance (RT_OPT_TUNE bit 6) against the default 4-wave one on the final kernel.
set -u
mkdir -p gpurun_out/w3; export TMPDIR=/tmp
O=gpurun_out/w3
L=raytracinginoneweekendinrust_amd/_lib/librtamd.so
{
for c in C3 C1; do for t in 0 64 0 64; do
  echo "== $c tune=$t"; RT_TUNE=$t timeout -k 10 200 python -u tools/ab_time.py --config $c --spp 100 --reps 3 $L || exit 1
done; done
} > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
