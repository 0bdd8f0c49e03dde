set -u
mkdir -p gpurun_out/r02h; export TMPDIR=/tmp
O=gpurun_out/r02h
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for t in 0 64; do
RT_TUNE=$t timeout -k 10 300 python3 tools/render_once.py --config C3 --reps 2 >> $O/c3_w.log 2>&1 || exit 1
RT_TUNE=$t timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w$t -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 100 > $O/w$t.log 2>&1; echo "pmc $t rc=$?"
done
grep -v amdgpu $O/c3_w.log
