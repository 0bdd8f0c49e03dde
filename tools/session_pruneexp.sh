set -u
mkdir -p gpurun_out/pruneexp; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/pruneexp
timeout -k 10 200 python3 tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd.so > $O/c4_base.log 2>&1 || exit $?
RT_TUNE=1048576 timeout -k 10 200 python3 tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd.so > $O/c4_pruneall.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/ab_time.py --config C4 --spp 50 --reps 3 $L/librtamd.so >> $O/c4_base.log 2>&1 || exit $?
grep -v amdgpu $O/c4_base.log $O/c4_pruneall.log
