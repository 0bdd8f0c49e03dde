set -u
mkdir -p gpurun_out/agroup2; export TMPDIR=/tmp
O=gpurun_out/agroup2
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for n in 2 4 8; do timeout -k 10 200 python3 tools/shard_time.py --config C3 --n $n >> $O/c3.log 2>&1 || exit 1; done
for c in "C1 50" "C2 500" "C4 1000" "C5 2000" "C3 63" "C3 125" "C3 250"; do set -- $c; timeout -k 10 200 python3 tools/render_once.py --config $1 --spp $2 --reps 2 >> $O/cfg.log 2>&1 || exit 1; done
grep -v amdgpu $O/c3.log $O/cfg.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-250
