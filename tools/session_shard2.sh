set -u
mkdir -p gpurun_out/shard2; export TMPDIR=/tmp
O=gpurun_out/shard2
timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 63 --reps 3 >> $O/c3.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 125 --reps 3 >> $O/c3.log 2>&1 || exit 1
RT_GROUP=4 timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 >> $O/c3.log 2>&1 || exit 1
RT_GROUP=8 timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 >> $O/c3.log 2>&1 || exit 1
RT_GROUP=32 timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 >> $O/c3.log 2>&1 || exit 1
grep -v amdgpu $O/c3.log
