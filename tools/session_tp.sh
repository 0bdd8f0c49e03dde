set -u
mkdir -p gpurun_out/tp; export TMPDIR=/tmp
O=gpurun_out/tp
L=raytracinginoneweekendinrust_amd/_lib
for spp in 63 500; do RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 200 python3 tools/region_profile.py --config C3 --spp $spp > $O/c3_$spp.log 2>&1 || exit 1; grep -E "wave_times|trace" $O/c3_$spp.log; done
