set -u
mkdir -p gpurun_out/shardprof; export TMPDIR=/tmp
O=gpurun_out/shardprof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/shard_time.py --config C3 --n 8 --reps 4 > $O/shard.log 2>&1 || exit 1
cat $O/shard.log | grep shard
python3 - <<'PY'
import csv,glob
rows=[r for f in glob.glob('gpurun_out/shardprof/prof/*kernel_trace.csv') for r in csv.DictReader(open(f))]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in rows:
    n=r['Kernel_Name']
    if 'trace_samples' in n or 'resolve' in n:
        print(n[:45], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6, r['Grid_Size'])
PY
