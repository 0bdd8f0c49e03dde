set -u
L=raytracinginoneweekendinrust_amd/_lib
mkdir -p gpurun_out/s9
timeout -k 10 300 python3 -u bench.py > gpurun_out/s9/bench_C3.log 2>&1 || exit 1
tail -1 gpurun_out/s9/bench_C3.log | cut -c1-400
RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 300 python3 -u tools/region_profile.py --config C3 --spp 64 > gpurun_out/s9/regions_c3_64spp.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 > gpurun_out/s9/shard8.log 2>&1 || exit 1
cat gpurun_out/s9/shard8.log | grep -v amdgpu.ids
