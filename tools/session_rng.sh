set -u
mkdir -p gpurun_out/rng; export TMPDIR=/tmp
L=raytracinginoneweekendinrust_amd/_lib; O=gpurun_out/rng
timeout -k 10 300 python3 tools/ab_time.py --config C3 --spp 100 --reps 3 $L/librtamd.so $L/librtamd_phx2.so $L/librtamd_pref.so $L/librtamd.so $L/librtamd_pref.so > $O/c3.log 2>&1 || exit $?
cat $O/c3.log
for c in "C4 50" "C5 200" "C2 64"; do set -- $c
timeout -k 10 300 python3 tools/ab_time.py --config $1 --spp $2 --reps 3 $L/librtamd.so $L/librtamd_pref.so $L/librtamd.so $L/librtamd_pref.so > $O/$1.log 2>&1 || exit $?
cat $O/$1.log; done
