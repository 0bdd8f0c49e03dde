set -u
mkdir -p gpurun_out/r02n; export TMPDIR=/tmp
O=gpurun_out/r02n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/shard_time.py --config C3 --n 8 --reps 5 > $O/shard8_C3.log 2>&1 || exit 1; grep shard $O/shard8_C3.log
