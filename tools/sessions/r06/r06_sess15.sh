#!/usr/bin/env bash
# Round 6, call 15: the bench half of the evidence set for the final library (tools/final_evidence.sh bench:
# one line per config, the driver-style C3 line, the whole GPU suite, smoke()), then the hand-over counts
# and frame times of C4 and C3 (tools/replay_count.py).
set -u
cd "$(dirname "$0")/../../.."
ROUND=r06 bash tools/final_evidence.sh bench && \
    timeout -k 10 400 python3 -u tools/replay_count.py C4:50 C4 C3:100 > gpurun_out/final_r06/replay_count.log 2>&1
