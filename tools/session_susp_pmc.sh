set -u
mkdir -p gpurun_out/spmc; export TMPDIR=/tmp
O=gpurun_out/spmc
for v in librtamd librtamd_suspall; do
RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/$v.so timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/$v -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 32 > $O/$v.log 2>&1; rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
