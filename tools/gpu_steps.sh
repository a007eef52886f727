#!/bin/bash
# Run GPU steps given as NAME=COMMAND arguments in order, each under its own time limit
# (STEP_TIMEOUT, default 600 s), output to gpurun_out/<NAME>.log.  A fault, abort or timeout
# (exit status other than 0/1) stops the script: no further GPU step runs after it.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%=*}"
    cmd="${spec#*=}"
    echo "== $name: $cmd"; date
    timeout -k 10 "${STEP_TIMEOUT:-600}" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    tail -4 "gpurun_out/$name.log"
    case "$rc" in
        0|1) ;;
        *) echo "STOP: $name exited $rc -- no further GPU steps"; exit "$rc" ;;
    esac
done
echo "== done"; date
