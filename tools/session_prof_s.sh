set -u
mkdir -p gpurun_out/prof_s; export TMPDIR=/tmp
O=gpurun_out/prof_s
L=raytracinginoneweekendinrust_amd/_lib
for c in C3 C4; do
for v in prof prof_s8; do
RT_LIBRARY=$L/librtamd_$v.so timeout -k 10 200 python3 tools/region_profile.py --config $c --spp 32 > $O/${c}_$v.log 2>&1; rc=$?; echo "$c $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done; done
