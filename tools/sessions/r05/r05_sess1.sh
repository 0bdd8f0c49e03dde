set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh trip 'C3:100 C1 C2:64 C5:200' $L/librtamd.so:migrate=0 $L/librtamd_trip0.so:migrate=0 $L/librtamd_nosort1.so:migrate=0 $L/librtamd_nosort2.so:migrate=0 || exit 1
bash tools/ab_session.sh mig 'C3:100 C1' $L/librtamd.so:migrate=0 $L/librtamd.so:migrate=8 $L/librtamd.so:migrate=16 $L/librtamd.so:migrate=32 || exit 1
mkdir -p gpurun_out/shard
for m in 0 16 0 16; do RT_MIGRATE=$m timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 5 >> gpurun_out/shard/c3_migrate_$m.log 2>&1 || exit 1; tail -n 2 gpurun_out/shard/c3_migrate_$m.log; done
bash tools/ab_session.sh tripc4 'C4:50' $L/librtamd.so:migrate=0 $L/librtamd_trip0.so:migrate=0 || exit 1
mkdir -p gpurun_out/c4cache && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/c4cache/pmc -o c4 --output-format csv -- python3 bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c4cache/pmc.log 2>&1; echo pmc rc=$?
