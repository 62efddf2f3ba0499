#!/bin/bash
# Runs GPU steps on the gpurun box, each under its own time limit; stops at the first
# crash/abort/timeout (exit codes other than 0/1/2/5), continues after ordinary test
# failures so one call yields tests + smoke + bench.
#   usage: tools/gpu_check.sh "<name>:<seconds>:<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"
    secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/steps.log
    tail -n 5 "gpurun_out/$name.log"
    case $rc in
        0|1|2|5) ;;
        *) echo "fatal rc=$rc in $name: stopping"; exit "$rc" ;;
    esac
done
