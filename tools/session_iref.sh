set -u
mkdir -p gpurun_out/iref; export TMPDIR=/tmp
O=gpurun_out/iref
L=raytracinginoneweekendinrust_amd/_lib
RT_LAUNCH_LOG=1 timeout -k 10 200 python3 tools/ab_time.py --config C3 --spp 8 --reps 1 $L/librtamd_iref.so > $O/log.log 2>&1 || { cat $O/log.log; exit 1; }
grep "rt:" $O/log.log | head -3
for c in C3 C1 C2 C5; do timeout -k 10 300 python3 tools/ab_time.py --config $c --reps 2 $L/librtamd.so $L/librtamd_iref.so $L/librtamd.so $L/librtamd_iref.so > $O/ab_$c.log 2>&1 || { cat $O/ab_$c.log; exit 1; }; echo "== $c"; tail -5 $O/ab_$c.log; done
