set -u
mkdir -p gpurun_out/r02m; export TMPDIR=/tmp
O=gpurun_out/r02m
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1; rc=$?; tail -3 $O/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for c in C3 C1; do timeout -k 10 200 python -u tools/shard_time.py --config $c --n 8 --reps 5 > $O/shard8_$c.log 2>&1 || exit 1; grep shard $O/shard8_$c.log; done
bash tools/profile_r02.sh final3
