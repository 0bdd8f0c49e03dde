set -u
mkdir -p gpurun_out/sched2; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/sched2
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_mcdef.so $L/librtamd_mcilp.so $L/librtamd.so $L/librtamd_mcdef.so $L/librtamd_mcilp.so > $O/c3.log 2>&1 || exit $?
grep -v amdgpu $O/c3.log
