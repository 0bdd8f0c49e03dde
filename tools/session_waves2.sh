set -u
mkdir -p gpurun_out/waves2; export TMPDIR=/tmp
O=gpurun_out/waves2
L=raytracinginoneweekendinrust_amd/_lib
for a in "--spp 63" "--shard 8" "--shard 8 --spp 250"; do n=$(echo $a | tr -d ' -'); RT_LIBRARY=$L/librtamd_prof.so timeout -k 10 200 python3 tools/region_profile.py --config C3 $a > $O/c3_$n.log 2>&1 || exit 1; echo "== $a"; grep -E "wave_times|trace" $O/c3_$n.log; done
