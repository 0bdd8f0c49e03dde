set -u
mkdir -p gpurun_out/regions; export TMPDIR=/tmp
O=gpurun_out/regions; L=raytracinginoneweekendinrust_amd/_lib
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 200 python3 tools/region_profile.py --config C3 --spp 64 > $O/c3_64.log 2>&1; rc=$?; cat $O/c3_64.log; exit $rc
