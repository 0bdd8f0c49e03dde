set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh uni 'C4:50 C5:200 C3:100 C1 C2:64' $L/librtamd.so $L/librtamd_cube0.so $L/librtamd_mark0.so $L/librtamd_base0.so $L/librtamd_urect0.so $L/librtamd_uentry0.so || exit 1
bash tools/ab_session.sh w4 'C4:50 C1' $L/librtamd.so $L/librtamd.so:tune=0x400000 || exit 1
mkdir -p gpurun_out/pipe gpurun_out/regions
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 5 > gpurun_out/pipe/serial.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 10 --pipeline > gpurun_out/pipe/pipelined.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pipe/*.log
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C3 --spp 64 > gpurun_out/regions/regions_c3_64spp.log 2>&1 || exit 1
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C4 --spp 16 > gpurun_out/regions/regions_c4_16spp.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pipe/gpu_tests.log 2>&1; echo gpu rc=$?; tail -3 gpurun_out/pipe/gpu_tests.log
