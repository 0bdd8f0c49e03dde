# The 3-wave default for the BVH-only and triangle presets: GPU suite, smoke, bench lines for C1, C4, C3.
set -u
mkdir -p gpurun_out/r02p; export TMPDIR=/tmp
O=gpurun_out/r02p
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
for c in C1 C4 C3; do
timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.log 2>&1; rc=$?; echo "$c rc=$rc"; grep '^{' $O/bench_$c.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
