set -u
mkdir -p gpurun_out/sched; export TMPDIR=/tmp
O=gpurun_out/sched
L=raytracinginoneweekendinrust_amd/_lib
for c in "C3 100 3" "C2 64 3" "C1 200 3"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps $3 $L/librtamd.so $L/librtamd_sdef.so $L/librtamd_silp.so $L/librtamd_socc.so $L/librtamd.so > $O/ab_$1.log 2>&1; rc=$?; echo "ab $1 rc=$rc"; grep -v amdgpu $O/ab_$1.log; [ $rc -eq 0 ] || exit $rc
done
