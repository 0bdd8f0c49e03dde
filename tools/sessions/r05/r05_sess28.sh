set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh mtlds 'C5 C3:100 C4 C2:64' $L/librtamd.so $L/librtamd_r5f.so || exit 1
