# Round-2 closing evidence: rocprof trace + PMC passes of the final kernel, then one bench line per config.
set -u
bash tools/profile_r02.sh final5 || exit 1
bash tools/session_configs.sh
