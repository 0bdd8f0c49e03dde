set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh grp 'C4 C2 C5' $L/librtamd.so:group=16 $L/librtamd.so:group=24 || exit 1
