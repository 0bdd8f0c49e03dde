set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh stride 'C3' $L/librtamd.so $L/librtamd_stride.so $L/librtamd_stride.so:0x800000 || exit 1
