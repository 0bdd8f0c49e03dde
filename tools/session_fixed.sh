set -u
mkdir -p gpurun_out/fixed; export TMPDIR=/tmp
O=gpurun_out/fixed
run() { timeout -k 10 200 env "$@" > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }; grep -h "shard 0/1" $O/tmp.log | sed "s/^/$1 $4 $5 /"; }
run RT_GROUP=0 python3 tools/shard_time.py --spp 63 --n 1 --reps 4
run RT_GROUP=16 python3 tools/shard_time.py --spp 63 --n 1 --reps 4
run RT_GROUP=4 python3 tools/shard_time.py --spp 63 --n 1 --reps 4
run RT_GROUP=4 python3 tools/shard_time.py --spp 500 --n 1 --reps 2
run RT_GROUP=0 python3 tools/shard_time.py --spp 125 --n 1 --reps 4
run RT_GROUP=0 python3 tools/shard_time.py --spp 250 --n 1 --reps 3
run RT_GROUP=0 python3 tools/shard_time.py --spp 16 --n 1 --reps 6
