set -u
mkdir -p gpurun_out/mlate; export TMPDIR=/tmp
O=gpurun_out/mlate
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_mlate.so $L/librtamd.so $L/librtamd_mlate.so > $O/ab_c3.log 2>&1; rc=$?; echo "ab c3 rc=$rc"; grep -v amdgpu $O/ab_c3.log
[ $rc -eq 0 ] || exit $rc
RT_LIBRARY=$L/librtamd_mlate.so timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 100 > $O/w.log 2>&1; echo "pmc rc=$?"
RT_LIBRARY=$L/librtamd_mlate.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
