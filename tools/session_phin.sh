set -u
mkdir -p gpurun_out/phin; export TMPDIR=/tmp
O=gpurun_out/phin
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_phin.so $L/librtamd.so $L/librtamd_phin.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
for c in "C2 64" "C5 200" "C4 50" "C1 50"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps 2 $L/librtamd.so $L/librtamd_phin.so > $O/ab_$1.log 2>&1; rc=$?; echo "ab $1 rc=$rc"; grep -v amdgpu $O/ab_$1.log; done
for v in librtamd librtamd_phin; do
RT_LIBRARY=$L/$v.so timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 32 > $O/w_$v.log 2>&1; echo "pmc $v rc=$?"
done
