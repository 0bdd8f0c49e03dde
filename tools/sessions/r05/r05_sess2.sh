set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh mig2 'C3:100 C1 C5:200' $L/librtamd.so:migrate=0 $L/librtamd.so:migrate=8 $L/librtamd.so:migrate=16 $L/librtamd.so:migrate=32 $L/librtamd.so:migrate=64 || exit 1
mkdir -p gpurun_out/shard2
for m in 0 16 64 0 16 64; do RT_MIGRATE=$m timeout -k 10 300 python3 -u tools/shard_time.py --config C3 --n 8 --reps 5 >> gpurun_out/shard2/c3_migrate_$m.log 2>&1 || exit 1; tail -n 2 gpurun_out/shard2/c3_migrate_$m.log; done
timeout -k 10 300 ./tools/markstein_check > gpurun_out/markstein_check.log 2>&1; echo markstein rc=$?; tail -3 gpurun_out/markstein_check.log
