set -u
mkdir -p gpurun_out/scal
for n in 2 4 8 16; do
  timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n $n --reps 4 --shard-only > gpurun_out/scal/serial_n$n.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n $n --reps 8 --pipeline --shard-only > gpurun_out/scal/pipelined_n$n.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --rank 5 --reps 4 --shard-only > gpurun_out/scal/serial_n8_rank5.log 2>&1 || exit 1
RT_GROUP=16 timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 > gpurun_out/scal/serial_n8_group16.log 2>&1 || exit 1
for f in gpurun_out/scal/*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
ROUND=r05 CFGS="C3 C1" bash tools/final_evidence.sh profiles
