set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh rrun 'C4 C5 C3:100' $L/librtamd.so $L/librtamd_base.so || exit 1
