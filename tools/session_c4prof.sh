set -u
mkdir -p gpurun_out/c4prof; export TMPDIR=/tmp
O=gpurun_out/c4prof
RT_LAUNCH_LOG=1 timeout -k 10 200 python3 tools/render_once.py --config C4 --spp 128 --reps 1 > $O/c4_128.log 2>&1 || exit 1
cat $O/c4_128.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o c4 --output-format csv -- python3 tools/render_once.py --config C4 --spp 128 --reps 1 > $O/prof.log 2>&1; echo "prof rc=$?"
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-250
