set -u
mkdir -p gpurun_out/r02i; export TMPDIR=/tmp
O=gpurun_out/r02i
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 tools/render_once.py --config C3 --spp 100 > $O/w.log 2>&1; echo "pmc rc=$?"
for c in "C1 200" "C2 64" "C4 50" "C5 200"; do set -- $c; timeout -k 10 200 python3 tools/render_once.py --config $1 --spp $2 --reps 2 >> $O/cfg.log 2>&1 || exit 1; done; grep -v amdgpu $O/cfg.log
