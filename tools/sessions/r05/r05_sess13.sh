set -u
mkdir -p gpurun_out/s13
for g in 1 2 4 8; do
  echo "guide $g" >> gpurun_out/s13/sweep.log
  RT_GUIDE=$g timeout -k 10 120 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --shard-only 2>&1 | grep -v amdgpu.ids >> gpurun_out/s13/sweep.log || exit 1
done
for gr in 2 8 16; do
  echo "group $gr" >> gpurun_out/s13/sweep.log
  RT_GROUP=$gr timeout -k 10 120 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --shard-only 2>&1 | grep -v amdgpu.ids >> gpurun_out/s13/sweep.log || exit 1
done
cat gpurun_out/s13/sweep.log
