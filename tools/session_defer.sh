set -u
mkdir -p gpurun_out/defer; export TMPDIR=/tmp
O=gpurun_out/defer
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_defer8.so $L/librtamd_defer16.so $L/librtamd_defer32.so $L/librtamd.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_time.py --config C4 --spp 50 --reps 2 $L/librtamd.so $L/librtamd_defer8.so $L/librtamd_defer16.so $L/librtamd_defer32.so > $O/ab_c4.log 2>&1; rc=$?; echo "ab c4 rc=$rc"; grep -v amdgpu $O/ab_c4.log
timeout -k 10 300 python3 tools/ab_time.py --config C1 --spp 200 --reps 3 $L/librtamd.so $L/librtamd_defer8.so $L/librtamd_defer16.so $L/librtamd_defer32.so > $O/ab_c1.log 2>&1; rc=$?; echo "ab c1 rc=$rc"; grep -v amdgpu $O/ab_c1.log
