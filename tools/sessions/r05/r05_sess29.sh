set -u
mkdir -p gpurun_out/s29
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_exec_join.py -q -x --timeout 240 --timeout-method thread > gpurun_out/s29/exec_join.log 2>&1 || { tail -30 gpurun_out/s29/exec_join.log; exit 1; }
tail -1 gpurun_out/s29/exec_join.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s29/smoke.log 2>&1 || { tail -20 gpurun_out/s29/smoke.log; exit 1; }
tail -1 gpurun_out/s29/smoke.log
