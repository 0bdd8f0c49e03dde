set -u
mkdir -p gpurun_out/guide; export TMPDIR=/tmp
O=gpurun_out/guide
run() { timeout -k 10 200 env "$@" > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }; grep -h "shard" $O/tmp.log | tail -1 | sed "s/^/$1 $2 $5 $6 /"; }
for gd in 2 4 8 16 32; do run RT_GROUP=0 RT_GUIDE=$gd python3 tools/shard_time.py --spp 63 --n 1 --reps 4; done
for gd in 8 16 32; do run RT_GROUP=16 RT_GUIDE=$gd python3 tools/shard_time.py --spp 63 --n 1 --reps 4; done
for gd in 2 8 16 32; do run RT_GROUP=0 RT_GUIDE=$gd python3 tools/shard_time.py --spp 500 --n 1 --reps 2; done
for gd in 8 32; do run RT_GROUP=32 RT_GUIDE=$gd python3 tools/shard_time.py --spp 500 --n 1 --reps 2; done
