# One bench line per BASELINE config (bench.py --config Cx, default steps/warmup), for DESIGN.md's table.
set -u
mkdir -p gpurun_out/configs; export TMPDIR=/tmp
O=gpurun_out/configs
for c in C1 C2 C3 C4 C5; do
timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.log 2>&1; rc=$?; echo "$c rc=$rc"; grep '^{' $O/bench_$c.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
done
