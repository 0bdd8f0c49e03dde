set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh mig3 'C3:100 C2:64 C5:200 C4:50 C1' $L/librtamd.so $L/librtamd_nomig.so || exit 1
mkdir -p gpurun_out/pipe2
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 5 --shard-only > gpurun_out/pipe2/serial.log 2>&1 || exit 1
for m in 0 16 32 64 0 16; do
  RT_MIGRATE=$m timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --shard-only >> gpurun_out/pipe2/pipelined_m$m.log 2>&1 || exit 1
done
RT_MIGRATE=16 timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --pipeline > gpurun_out/pipe2/pipelined_full_m16.log 2>&1 || exit 1
for f in gpurun_out/pipe2/*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
