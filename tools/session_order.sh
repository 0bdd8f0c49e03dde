set -u
mkdir -p gpurun_out/order; export TMPDIR=/tmp
O=gpurun_out/order
timeout -k 10 120 python -u tools/order_check.py > $O/check.log 2>&1 || exit 1
cat $O/check.log
for rep in 1 2; do
for t in 0 0x200000; do
  RT_TUNE=$t timeout -k 10 120 python -u tools/shard_time.py --config C3 --n 8 --reps 5 > $O/shard8_${t}_$rep.log 2>&1 || exit 1
  echo "tune=$t rep=$rep"; grep shard $O/shard8_${t}_$rep.log
done
done
