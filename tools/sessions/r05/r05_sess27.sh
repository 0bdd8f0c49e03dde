set -u
L=raytracinginoneweekendinrust_amd/_lib
mkdir -p gpurun_out/s27
bash tools/ab_session.sh c1grp 'C1' $L/librtamd.so $L/librtamd.so:group=1 $L/librtamd.so:group=2 $L/librtamd.so:guide=4 || exit 1
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C3 --spp 64 > gpurun_out/s27/regions_c3_64spp.log 2>&1 || exit 1
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C4 --spp 16 > gpurun_out/s27/regions_c4_16spp.log 2>&1 || exit 1
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C5 --spp 32 > gpurun_out/s27/regions_c5_32spp.log 2>&1 || exit 1
echo ok
