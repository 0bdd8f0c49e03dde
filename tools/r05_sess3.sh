set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh uni 'C4:50 C5:200 C3:100 C1 C2:64' $L/librtamd.so $L/librtamd_mark0.so $L/librtamd_base0.so $L/librtamd_urect0.so $L/librtamd_uentry0.so || exit 1
mkdir -p gpurun_out/pipe
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 5 > gpurun_out/pipe/serial.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 10 --pipeline > gpurun_out/pipe/pipelined.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pipe/*.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multiprocess.py -q --timeout 300 --timeout-method thread > gpurun_out/pipe/multiprocess_tests.log 2>&1; echo mp rc=$?; tail -3 gpurun_out/pipe/multiprocess_tests.log
