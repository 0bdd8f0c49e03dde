set -u
L=raytracinginoneweekendinrust_amd/_lib
mkdir -p gpurun_out/mf
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mf/gpu_parity.log 2>&1 || { tail -30 gpurun_out/mf/gpu_parity.log; exit 1; }
tail -3 gpurun_out/mf/gpu_parity.log
bash tools/ab_session.sh mf 'C3:100 C1' $L/librtamd.so $L/librtamd_mf0.so $L/librtamd_mfl16.so || exit 1
for v in "" _mf0 _mfl16; do
  RT_LIBRARY=$L/librtamd$v.so timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 6 --shard-only > gpurun_out/mf/shard8$v.log 2>&1 || exit 1
  RT_LIBRARY=$L/librtamd$v.so timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 6 --shard-only >> gpurun_out/mf/shard8$v.log 2>&1 || exit 1
done
for f in gpurun_out/mf/shard8*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
