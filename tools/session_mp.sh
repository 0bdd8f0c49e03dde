# Rehearsal of bench.py's N>1 path (one process per rank, gloo barriers, shared-memory gather)
# on a one-GPU box: two ranks share the GPU. Not a scaling measurement.
set -u
mkdir -p gpurun_out/mp; export TMPDIR=/tmp
O=gpurun_out/mp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $O/n2.log 2>&1; rc=$?; echo "n2 rc=$rc"; grep '^{' $O/n2.log | cut -c1-400; tail -5 $O/n2.log
