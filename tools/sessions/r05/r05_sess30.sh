set -u
mkdir -p gpurun_out/s30
for c in C4 C3 C5; do
RT_LAUNCH_LOG=1 timeout -k 10 120 python3 -u tools/render_once.py --config $c --spp 100 > gpurun_out/s30/launch_$c.log 2>&1 || exit 1
done
grep -h "replayed\|trace_samples\|kernel" gpurun_out/s30/launch_*.log | grep -v amdgpu
