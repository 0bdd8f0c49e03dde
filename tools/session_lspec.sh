set -u
mkdir -p gpurun_out/lspec; export TMPDIR=/tmp
O=gpurun_out/lspec
L=raytracinginoneweekendinrust_amd/_lib
for c in "C3 100 3" "C1 200 3" "C4 50 2"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps $3 $L/librtamd_base2.so $L/librtamd_lspec.so $L/librtamd_base2.so $L/librtamd_lspec.so > $O/ab_$1.log 2>&1; rc=$?; echo "ab $1 rc=$rc"; grep -v amdgpu $O/ab_$1.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
