set -u
mkdir -p gpurun_out/s19
export TMPDIR=/tmp
RT_TUNE=0x20000 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/s19/tr -o ns3 -- python3 -u tools/shard_time.py --config C3 --n 8 --reps 9 --pipeline --handles 3 --shard-only > gpurun_out/s19/run.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/s19/run.log | grep shard
