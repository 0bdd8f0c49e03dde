#!/usr/bin/env bash
# Round 6, the evidence set for a final library through tools/final_evidence.sh: `profiles` = the rocprofv3
# kernel trace + PMC passes of every config and the PMC summaries (profiles/r06/pmc_*_C*.json); `bench` =
# one bench line per config, the driver-style C3 line, the GPU suite (multi-process tests included) and
# smoke(). Calls 10/11 ran it on a15b17a (md5 a50038f8...), calls 14/15 on 1e223779 (the fast-kernel
# zero-direction rule, non-temporal sample-buffer stores in the BVH presets only), calls 18/19 on 81d8c5fe (the NaN-t_max leaf scan).
set -u
cd "$(dirname "$0")/../../.."
ROUND=r06 bash tools/final_evidence.sh "${1:-profiles}"
