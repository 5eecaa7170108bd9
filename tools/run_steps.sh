#!/bin/bash
# Ad-hoc GPU-box step list for one gpurun call: each line of the file given as
# $1 is one command, run under its own time limit (the first field, seconds);
# the first failure ends the script (no GPU work after a failure).
#   tools/run_steps.sh STEPFILE
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
while IFS= read -r line; do
    [ -z "$line" ] && continue
    case "$line" in \#*) continue ;; esac
    t=${line%% *}
    cmd=${line#* }
    echo "[run_steps] $(date +%T) $cmd"
    timeout -k 10 "$t" bash -o pipefail -c "$cmd" || { echo "[run_steps] FAILED ($?): $cmd"; exit 1; }
done < "$1"
echo "[run_steps] done $(date +%T)"
