set -u
mkdir -p gpurun_out/replay; export TMPDIR=/tmp
O=gpurun_out/replay
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log
find $O/prof -name '*kernel_stats.csv' -exec cut -c1-60,300- {} \; | cut -d, -f1-6 | head -8 || true
for n in 8 4; do timeout -k 10 200 python3 tools/shard_time.py --config C3 --n $n --rank 0 --reps 3 > $O/shard_$n.log 2>&1 || exit 1; tail -2 $O/shard_$n.log; done
