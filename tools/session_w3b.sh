# The 3-wave instances (RT_OPT_TUNE bit 6) against the default choice, per config at its own size/spp
# (C3 at 100 spp, C4 at 50 spp, C5 at 200 spp: the same per-sample work).
set -u
mkdir -p gpurun_out/w3; export TMPDIR=/tmp
O=gpurun_out/w3
L=raytracinginoneweekendinrust_amd/_lib/librtamd.so
{
for cs in "C1 50" "C2 64" "C4 50" "C5 200"; do set -- $cs; for t in 0 64 0 64; do
  echo "== $1 tune=$t"; RT_TUNE=$t timeout -k 10 200 python -u tools/ab_time.py --config $1 --spp $2 --reps 3 $L || exit 1
done; done
} > $O/ab2.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab2.log; exit $rc
