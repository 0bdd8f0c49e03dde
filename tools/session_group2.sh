set -u
mkdir -p gpurun_out/group2; export TMPDIR=/tmp
O=gpurun_out/group2
for g in 8 12 14 16; do RT_GROUP=$g timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 250 --reps 2 >> $O/spp250.log 2>&1 || exit 1; done
for g in 4 5 8; do RT_GROUP=$g timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 100 --reps 2 >> $O/spp100.log 2>&1 || exit 1; done
for g in 8 14 16; do RT_GROUP=$g timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 2 --reps 2 >> $O/shard2.log 2>&1 || exit 1; done
for g in 4 7 8; do RT_GROUP=$g timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 4 --reps 2 >> $O/shard4.log 2>&1 || exit 1; done
grep -v amdgpu $O/*.log | grep -v "shard 0/1"
