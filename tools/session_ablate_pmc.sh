# VALU instructions per region on C3 (32 spp): the ablation build runs one region twice
# (RT_TUNE bit), so the counter deltas against the plain run price that region.
set -u
mkdir -p gpurun_out/abl; export TMPDIR=/tmp
O=gpurun_out/abl
L=raytracinginoneweekendinrust_amd/_lib/librtamd_ablate.so
for t in 0 256 512 1024 2048 4096; do
RT_LIBRARY=$L RT_TUNE=$t timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/t$t -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 32 > $O/t$t.log 2>&1; rc=$?; echo "tune $t rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
