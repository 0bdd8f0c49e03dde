set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd_base.so $L/librtamd.so $L/librtamd_noinl.so $L/librtamd_base.so > gpurun_out/ab1.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab1.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/par1.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/par1.log
