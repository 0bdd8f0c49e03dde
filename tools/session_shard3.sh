set -u
mkdir -p gpurun_out/shard3; export TMPDIR=/tmp
O=gpurun_out/shard3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o sh --output-format csv -- python3 tools/shard_time.py --config C3 --n 8 > $O/prof.log 2>&1; echo "prof rc=$?"
grep -v amdgpu $O/prof.log | grep shard
