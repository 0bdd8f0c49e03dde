set -u
mkdir -p gpurun_out; export TMPDIR=/tmp; rm -f gpurun_out/reference_images.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; grep '^{' gpurun_out/bench.log
bash tools/profile_r02.sh r02
