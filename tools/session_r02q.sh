# RT_SUSPEND 24: GPU suite, smoke, bench lines for C4 and C3 (round-end rehearsal of the final tree).
set -u
mkdir -p gpurun_out/r02q; export TMPDIR=/tmp
O=gpurun_out/r02q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
for c in C4 C3; do
timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.log 2>&1; rc=$?; echo "$c rc=$rc"; grep '^{' $O/bench_$c.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
