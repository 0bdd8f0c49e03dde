set -u
mkdir -p gpurun_out/s14
run() { # n group
  echo "n $1 group $2" >> gpurun_out/s14/sweep.log
  RT_GROUP=$2 timeout -k 10 120 python3 -u tools/shard_time.py --config C3 --n $1 --reps 3 --shard-only 2>&1 | grep -v amdgpu.ids >> gpurun_out/s14/sweep.log || exit 1
}
for g in 6 8 10 12 14; do run 8 $g; done
for g in 8 12 16 20 24 32; do run 1 $g; done
for g in 8 12 16 24; do run 2 $g; done
for g in 6 8 12 16; do run 4 $g; done
for g in 4 6 8; do run 16 $g; done
cat gpurun_out/s14/sweep.log
