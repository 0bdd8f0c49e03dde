set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh grp2 'C5 C4 C3' $L/librtamd.so:group=24 $L/librtamd.so:group=32 $L/librtamd.so:group=48 $L/librtamd.so:group=64 || exit 1
