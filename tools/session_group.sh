set -u
mkdir -p gpurun_out/group; export TMPDIR=/tmp
O=gpurun_out/group
for g in 1 2 4 8 16; do RT_GROUP=$g timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 --reps 2 >> $O/shard.log 2>&1 || exit 1; done
for g in 2 4 8 16; do RT_GROUP=$g timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 63 --reps 2 >> $O/spp63.log 2>&1 || exit 1; done
for g in 8 16 32; do RT_GROUP=$g timeout -k 10 200 python3 tools/render_once.py --config C3 --reps 2 >> $O/spp500.log 2>&1 || exit 1; done
grep -v amdgpu $O/*.log | grep -v "shard 0/1"
