set -u
mkdir -p gpurun_out/chunks; export TMPDIR=/tmp
O=gpurun_out/chunks
for mb in 0 3000 1500 700; do RT_SAMPLE_BUFFER_MB=$mb RT_LAUNCH_LOG=1 timeout -k 10 200 python3 tools/render_once.py --config C3 --reps 2 >> $O/c3.log 2>&1 || exit 1; done
for spp in 32 250 1000; do timeout -k 10 200 python3 tools/render_once.py --config C3 --spp $spp --reps 2 >> $O/c3.log 2>&1 || exit 1; done
grep -v amdgpu $O/c3.log | grep -v "features"
