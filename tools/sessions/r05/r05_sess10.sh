set -u
mkdir -p gpurun_out/s10
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 2 --spp 4000 > gpurun_out/s10/shard8_4000.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --spp 1000 --shard-only > gpurun_out/s10/shard8_1000.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --spp 250 > gpurun_out/s10/shard8_250.log 2>&1 || exit 1
for f in gpurun_out/s10/*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
