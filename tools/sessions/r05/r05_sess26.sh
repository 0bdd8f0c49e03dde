set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh mrcp 'C5 C3:100' $L/librtamd.so $L/librtamd_mrcp.so || exit 1
