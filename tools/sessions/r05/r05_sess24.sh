set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh sent 'C4 C5 C3:100 C1 C2:64' $L/librtamd.so $L/librtamd_rr.so || exit 1
