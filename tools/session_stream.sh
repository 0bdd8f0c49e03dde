set -u
mkdir -p gpurun_out/stream; export TMPDIR=/tmp
O=gpurun_out/stream
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "streaming" > $O/par.log 2>&1; rc=$?; tail -3 $O/par.log; [ $rc -eq 0 ] || exit 1
for t in 0 0x20000; do RT_TUNE=$t timeout -k 10 200 python3 tools/shard_time.py --config C3 --n 8 --reps 4 > $O/shard_$t.log 2>&1 || { cat $O/shard_$t.log; exit 1; }; sed "s/^/tune=$t /" $O/shard_$t.log | grep shard; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/shard_time.py --config C3 --n 8 --reps 2 > $O/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
rows=[r for f in glob.glob('gpurun_out/stream/prof/*kernel_trace.csv') for r in csv.DictReader(open(f))]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t0=None
for r in rows:
    n=r['Kernel_Name']
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    if 'trace_samples' in n or 'resolve' in n:
        if t0 is None or 'trace_samples<0' in n: t0=s
        print(n[29:52], 'start', round((s-t0)/1e6,3), 'end', round((e-t0)/1e6,3))
PY
