set -u
mkdir -p gpurun_out/r02f; export TMPDIR=/tmp
O=gpurun_out/r02f
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for spp in 128 1000; do RT_LAUNCH_LOG=1 timeout -k 10 300 python3 tools/render_once.py --config C4 --spp $spp --reps 1 >> $O/c4.log 2>&1 || exit 1; done
timeout -k 10 300 python3 tools/render_once.py --config C5 --reps 1 >> $O/c4.log 2>&1 || exit 1
grep -v amdgpu.ids $O/c4.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cut -c1-400 $O/bench.log | tail -1
