set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh sw 'C4 C3 C5' $L/librtamd.so $L/librtamd_sw1k.so $L/librtamd_sw2k.so || exit 1
