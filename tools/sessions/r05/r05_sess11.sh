set -u
L=raytracinginoneweekendinrust_amd/_lib
mkdir -p gpurun_out/s11
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C3 --shard 8 > gpurun_out/s11/regions_c3_shard8.log 2>&1 || exit 1
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C3 > gpurun_out/s11/regions_c3_full.log 2>&1 || exit 1
echo done
