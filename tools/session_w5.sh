set -u
mkdir -p gpurun_out/w5; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/w5
RT_LAUNCH_LOG=1 timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_w5.so $L/librtamd_pinl.so $L/librtamd.so $L/librtamd_w5.so $L/librtamd_pinl.so > $O/c3.log 2>&1 || exit $?
grep -v "^\[rt\] fast" $O/c3.log | grep -v amdgpu; grep "^\[rt\]" $O/c3.log | sort | uniq -c | head
timeout -k 10 300 python3 tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd.so $L/librtamd_w5.so $L/librtamd_pinl.so $L/librtamd.so $L/librtamd_w5.so $L/librtamd_pinl.so > $O/c4.log 2>&1 || exit $?
cat $O/c4.log
