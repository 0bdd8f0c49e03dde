set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh w4c4 'C4' $L/librtamd.so $L/librtamd.so:0x400000 || exit 1
