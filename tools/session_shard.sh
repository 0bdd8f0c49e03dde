set -u
mkdir -p gpurun_out/shard; export TMPDIR=/tmp
O=gpurun_out/shard
for n in 2 4 8; do timeout -k 10 200 python3 tools/shard_time.py --config C3 --n $n >> $O/c3.log 2>&1 || exit 1; done
timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 --rank 7 >> $O/c3.log 2>&1 || exit 1
grep -v amdgpu $O/c3.log
