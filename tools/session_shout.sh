set -u
mkdir -p gpurun_out/shout; export TMPDIR=/tmp
O=gpurun_out/shout
L=raytracinginoneweekendinrust_amd/_lib
for c in "C1 200 3" "C2 64 3" "C4 50 2" "C5 200 2"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps $3 $L/librtamd.so $L/librtamd_shout.so $L/librtamd.so $L/librtamd_shout.so > $O/ab_$1.log 2>&1; rc=$?; echo "ab $1 rc=$rc"; grep -v amdgpu $O/ab_$1.log; [ $rc -eq 0 ] || exit $rc
done
