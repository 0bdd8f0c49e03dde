set -u
ROUND=r05 CFGS="C2 C4 C5" bash tools/final_evidence.sh profiles || exit 1
mkdir -p gpurun_out/ovl && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ovl/trace -o ovl --output-format csv -- python3 tools/shard_time.py --config C3 --n 8 --reps 6 --pipeline --shard-only > gpurun_out/ovl/run.log 2>&1; echo ovl rc=$?
