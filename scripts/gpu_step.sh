#!/bin/bash
# usage: scripts/gpu_step.sh NAME TIMEOUT_S cmd...   (run on the GPU box)
# Runs one GPU step under its own time limit, logs to gpurun_out/NAME.log.
# Exit status 0/1 (pass / test failures) lets the caller continue; anything
# else (fault, abort, segfault, timeout) is passed through so the chain stops.
set -u
name=$1; shift
lim=$1; shift
mkdir -p gpurun_out
timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$name] rc=$rc"
tail -n 5 "gpurun_out/$name.log"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then exit 0; fi
exit $rc
