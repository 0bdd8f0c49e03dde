#!/usr/bin/env bash
# Round 6, call 24: one rank's share of the 8-GPU C3 step on the round's final library (81d8c5fe), timed on one
# MI355X (tools/shard_time.py): the whole frame and shard 0 of 8 serial, shard 0 and 5 of 8 with frames in flight
# (the N > 1 bench's mode), and shard 0 of 2 and of 4 pipelined.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s24
mkdir -p "$OUT"
r() {
    echo "== python3 -u tools/shard_time.py $*" >> "$OUT/shard.log"
    timeout -k 10 300 python3 -u tools/shard_time.py "$@" 2>&1 | grep -v amdgpu.ids >> "$OUT/shard.log" || exit 1
}
r --config C3 --n 8 --reps 4
r --config C3 --n 8 --reps 12 --pipeline --shard-only
r --config C3 --n 8 --rank 5 --reps 12 --pipeline --shard-only
r --config C3 --n 4 --reps 8 --pipeline --shard-only
r --config C3 --n 2 --reps 6 --pipeline --shard-only
echo "== done" >> "$OUT/shard.log"
