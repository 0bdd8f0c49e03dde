set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh stop 'C3:100 C2:64 C1 C4' $L/librtamd.so $L/librtamd_se.so || exit 1
