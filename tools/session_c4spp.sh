set -u
mkdir -p gpurun_out/c4spp; export TMPDIR=/tmp
O=gpurun_out/c4spp
R="python3 tools/render_once.py --config C4"
for spp in 50 128 255 256 500; do timeout -k 10 200 $R --spp $spp --reps 2 >> $O/c4.log 2>&1 || exit 1; done
RT_GROUP=8 timeout -k 10 200 $R --spp 500 --reps 2 >> $O/c4.log 2>&1 || exit 1
RT_GROUP=4 timeout -k 10 200 $R --spp 500 --reps 2 >> $O/c4.log 2>&1 || exit 1
RT_GROUP=16 timeout -k 10 200 $R --spp 50 --reps 2 >> $O/c4.log 2>&1 || exit 1
for g in 4 8 16; do RT_GROUP=$g timeout -k 10 200 python3 tools/render_once.py --config C3 --spp 500 --reps 2 >> $O/c3.log 2>&1 || exit 1; done
cat $O/c4.log $O/c3.log | grep -v amdgpu.ids
