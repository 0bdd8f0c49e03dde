set -u
mkdir -p gpurun_out/s17
for n in 2 4 8 16; do
  timeout -k 10 200 python3 -u tools/shard_time.py --config C3 --n $n --reps 4 $( [ $n = 2 ] || echo --shard-only ) 2>&1 | grep -v amdgpu.ids >> gpurun_out/s17/series.log || exit 1
done
timeout -k 10 200 python3 -u tools/shard_time.py --config C3 --n 8 --rank 5 --reps 4 --shard-only 2>&1 | grep -v amdgpu.ids >> gpurun_out/s17/series.log || exit 1
timeout -k 10 200 python3 -u tools/shard_time.py --config C3 --n 8 --reps 8 --pipeline --shard-only 2>&1 | grep -v amdgpu.ids >> gpurun_out/s17/series.log || exit 1
cat gpurun_out/s17/series.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/s17/bench_C3.log 2>&1 || exit 1
tail -1 gpurun_out/s17/bench_C3.log | cut -c1-300
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/s17/gpu_tests.log 2>&1 || { tail -30 gpurun_out/s17/gpu_tests.log; exit 1; }
tail -2 gpurun_out/s17/gpu_tests.log
