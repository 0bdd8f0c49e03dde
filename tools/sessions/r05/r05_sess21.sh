set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh geo 'C3:100' $L/librtamd.so $L/librtamd_geo.so || exit 1
