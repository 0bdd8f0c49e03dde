set -u
mkdir -p gpurun_out/stream2; export TMPDIR=/tmp
O=gpurun_out/stream2
L=raytracinginoneweekendinrust_amd/_lib
for t in 0 0x20000; do RT_TUNE=$t RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 200 python3 tools/region_profile.py --config C3 --shard 8 > $O/c3_$t.log 2>&1 || { tail $O/c3_$t.log; exit 1; }; echo "== tune $t"; grep -E "wave_times|trace|role_ev" $O/c3_$t.log; done
