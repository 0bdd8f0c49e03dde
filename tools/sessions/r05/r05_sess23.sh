set -u
mkdir -p gpurun_out/s23
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/s23/avail.txt 2>&1 || true
grep -o "SQC_[A-Z0-9_]*" gpurun_out/s23/avail.txt | sort -u > gpurun_out/s23/sqc_names.txt || true
B="python3 tools/render_once.py --config C3 --spp 32"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES -d gpurun_out/s23/ic -o c3 --output-format csv -- $B > gpurun_out/s23/ic.log 2>&1 || echo "ic rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_MISSES -d gpurun_out/s23/dc -o c3 --output-format csv -- $B > gpurun_out/s23/dc.log 2>&1 || echo "dc rc=$?"
B="python3 tools/render_once.py --config C4 --spp 32"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES -d gpurun_out/s23/ic4 -o c4 --output-format csv -- $B > gpurun_out/s23/ic4.log 2>&1 || echo "ic4 rc=$?"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/s23/parity.log 2>&1 || { tail -30 gpurun_out/s23/parity.log; exit 1; }
tail -1 gpurun_out/s23/parity.log
