set -u
mkdir -p gpurun_out/s18
r() { echo "== $*" >> gpurun_out/s18/pipe.log; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> gpurun_out/s18/pipe.log || exit 1; }
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --handles 2 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --handles 3 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --handles 4 --shard-only
export RT_TUNE=0x20000
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --handles 2 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --handles 3 --shard-only
cat gpurun_out/s18/pipe.log
