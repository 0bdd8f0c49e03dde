set -u
mkdir -p gpurun_out/s20
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_exec_join.py tests/test_gpu_multiprocess.py "tests/test_gpu_parity.py::test_streaming_replay_pass_matches_oracle" -q -x --timeout 300 --timeout-method thread > gpurun_out/s20/tests.log 2>&1 || { tail -30 gpurun_out/s20/tests.log; exit 1; }
tail -2 gpurun_out/s20/tests.log
r() { echo "== $*" >> gpurun_out/s20/pipe.log; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> gpurun_out/s20/pipe.log || exit 1; }
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 4 --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --reps 12 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 8 --rank 5 --reps 12 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 4 --reps 8 --pipeline --shard-only
r python3 -u tools/shard_time.py --config C3 --n 2 --reps 6 --pipeline
cat gpurun_out/s20/pipe.log
timeout -k 10 300 python3 -u bench.py --pipeline on > gpurun_out/s20/bench_pipe_n1.log 2>&1 || exit 1
tail -1 gpurun_out/s20/bench_pipe_n1.log | cut -c1-250
