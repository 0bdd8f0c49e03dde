set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh final 'C3:100 C4:50 C5:200 C1 C2:64' $L/librtamd.so $L/librtamd_base0.so $L/librtamd_mark0.so $L/librtamd_cube0.so || exit 1
mkdir -p gpurun_out/b4
timeout -k 10 300 python3 -u bench.py > gpurun_out/b4/bench_C3.log 2>&1 || exit 1
tail -c 600 gpurun_out/b4/bench_C3.log
