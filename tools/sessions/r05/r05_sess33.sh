set -u
L=raytracinginoneweekendinrust_amd/_lib
bash tools/ab_session.sh f64r 'C3:100 C3' $L/librtamd.so $L/librtamd_f64r.so || exit 1
