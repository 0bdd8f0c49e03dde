set -u
mkdir -p gpurun_out/s32
r() { echo "== $*" >> gpurun_out/s32/series.log; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> gpurun_out/s32/series.log || exit 1; }
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 4
r python3 -u tools/shard_time.py --config C3 --n 8 --rank 5 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --rank 5 --reps 12 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 4 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 4 --reps 8 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 2 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 2 --reps 6 --pipeline --shard-only
cat gpurun_out/s32/series.log
