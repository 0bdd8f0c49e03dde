set -u
mkdir -p gpurun_out/pad; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/pad
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_pt256.so $L/librtamd_pb32.so $L/librtamd.so $L/librtamd_pt256.so $L/librtamd_pb32.so > $O/c3.log 2>&1 || exit $?
cat $O/c3.log
