#!/usr/bin/env bash
# Round 6, calls 10-11: the evidence set for the round's final library (commit a15b17a, md5 a50038f8...):
# call 10 = the rocprofv3 kernel trace + PMC passes of every config and the PMC summaries
# (profiles/r06/pmc_*_C*.json); call 11 = one bench line per config, the driver-style C3 line,
# the GPU suite and smoke(). Both through tools/final_evidence.sh.
set -u
cd "$(dirname "$0")/../../.."
ROUND=r06 bash tools/final_evidence.sh "${1:-profiles}"
