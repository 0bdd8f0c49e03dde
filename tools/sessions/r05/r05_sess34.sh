set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh w4 'C1 C4:200' $L/librtamd.so $L/librtamd.so:0x400000 || exit 1
