#!/bin/bash
# Runs GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# A step that fails its tests (pytest rc 1) does not stop the rest; anything else (a time limit,
# an abort, a segfault, a GPU fault) ends the script there.
#   step <name> <seconds> <command...>
mkdir -p gpurun_out
step() {
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(tail -1 "gpurun_out/$name.log")"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "[$name] stopping: rc $rc"
        exit $rc
    fi
}
PYT="python -u -m pytest -v -s --timeout-method thread"
